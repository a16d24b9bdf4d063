"""Per-step times of the bench's graph-replayed step (config 4 shapes): is the
first step after the pre-timing synchronize slower than the rest?
    python tools/first_step.py [--videos N] [--steps K] [--spin MS]
--spin keeps the GPU busy with a dummy kernel loop for MS milliseconds right
before the timed steps (no host sync in between)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

def main():
    argv = sys.argv[1:]
    spin = 0.0
    if "--spin" in argv:
        i = argv.index("--spin"); spin = float(argv[i + 1]); del argv[i:i + 2]
    sys.argv = [sys.argv[0]] + argv + ["--no-cpu-baseline"]
    a = bench.parse()
    import torch
    from eks_amd import _lib
    dev = torch.device("cuda", 0)
    _lib.require_gpu()
    w = bench.workload_singleview(torch, a, dev, 0, 1, 4)
    step = w["step"]
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    x = torch.zeros(1 << 20, device=dev)
    for trial in range(3):
        torch.cuda.synchronize()
        if spin > 0:
            t = time.perf_counter()
            while (time.perf_counter() - t) * 1e3 < spin:
                x.mul_(1.0)
        t0 = time.perf_counter()
        ev[0].record()
        for k in range(a.steps):
            g.replay()
            ev[k + 1].record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        per = [ev[k].elapsed_time(ev[k + 1]) for k in range(a.steps)]
        print(f"trial {trial} spin {spin} ms: wall/step {wall / a.steps:.4f} ms, events: first "
              f"{per[0]:.4f} second {per[1]:.4f} median {sorted(per)[len(per) // 2]:.4f} "
              f"sum {sum(per):.3f} ms", flush=True)

main()
