"""Config-4 step time against the duty cycle: the step (eks_smooth: the two
algo-3 passes) timed with HIP events, followed by an idle GPU gap of G ms
(torch.cuda._sleep: one spinning wave), for G = 0 .. 3 ms.  If the chip is
power-limited at 100 % duty (the driver's back-to-back replays), the step
gets faster as the gap grows, at the same cycle count (the clock rises)."""
import os
import subprocess
import sys

sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

a = bench.parse()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
w = bench.workload_singleview(torch, a, dev, 0, 1, 4)
for _ in range(5):
    w["step"]()
torch.cuda.synchronize()


def power():
    try:
        out = subprocess.run(["amd-smi", "metric", "-p"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if "SOCKET_POWER" in line:
                return line.split(":")[1].strip()
    except Exception:
        pass
    return "?"


CYC_PER_MS = 100_000  # torch.cuda._sleep counts s_memtime-like cycles: calibrated below
# calibrate _sleep: cycles per ms on this box
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
torch.cuda._sleep(1_000_000)
e1.record()
torch.cuda.synchronize()
CYC_PER_MS = 1_000_000 / e0.elapsed_time(e1)
print(f"_sleep: {CYC_PER_MS:.0f} cycles per ms")
for gap in (0.0, 0.5, 1.0, 2.0, 3.0, 0.0):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(60)]
    for k, (s0, s1) in enumerate(ev):
        s0.record()
        w["step"]()
        s1.record()
        if gap > 0:
            torch.cuda._sleep(int(gap * CYC_PER_MS))
        if k == 40:
            torch.cuda.synchronize()
            pw = power()
    torch.cuda.synchronize()
    t = sorted(s0.elapsed_time(s1) for s0, s1 in ev[10:])
    print(f"gap {gap:.1f} ms: step median {t[len(t)//2]:.3f} ms  min {t[0]:.3f}  socket power after 40 steps {pw}")
