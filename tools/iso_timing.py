"""Step time of config 4 (or --videos N) isolated vs back to back: each
eks_smooth call timed with HIP events, (a) with 200 ms idle before each call,
(b) 30 calls back to back.  An idle gap lets the chip's clock recover
(MI355X_MICROARCH.md, DVFS give-back); the driver's bench times back-to-back
graph replays."""
import os
import sys
import time

sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

a = bench.parse()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
w = bench.workload_singleview(torch, a, dev, 0, 1, 4)
for _ in range(3):
    w["step"]()
torch.cuda.synchronize()


def timed(n, gap):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in ev:
        if gap:
            torch.cuda.synchronize()
            time.sleep(gap)
        e0.record()
        w["step"]()
        e1.record()
    torch.cuda.synchronize()
    return [e0.elapsed_time(e1) for e0, e1 in ev]


iso = timed(10, 0.2)
b2b = timed(30, 0)
iso2 = timed(10, 0.2)
print(f"isolated  (200 ms idle before each): {sorted(iso)[len(iso)//2]:.3f} ms median, min {min(iso):.3f}")
print(f"back to back (30 calls): first {b2b[0]:.3f}  median {sorted(b2b)[15]:.3f}  last {b2b[-1]:.3f}")
print(f"isolated again: {sorted(iso2)[len(iso2)//2]:.3f} ms median")
