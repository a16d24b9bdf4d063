"""Time eks_newton_filter (k_newton) on synthetic long trajectories."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time

import numpy as np
import torch

from eks_amd.newton_eks import newton_filter_batch

for Bn, T, r, n in [(1, 10000, 3, 4), (17, 10000, 3, 4), (1024, 10000, 3, 8), (17408, 10000, 2, 2)]:
    rng = np.random.default_rng(0)
    y = torch.randn(Bn, T, n, dtype=torch.float64, device="cuda")
    ev = torch.rand(Bn, T, n, dtype=torch.float64, device="cuda") + 0.1
    mu0 = np.zeros(r); S0 = np.eye(r); A = np.eye(r); E = np.eye(r) * 0.1
    Bm = rng.normal(size=(n, r))
    newton_filter_batch(y, ev, mu0, S0, A, Bm, E)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        q, st = newton_filter_batch(y, ev, mu0, S0, A, Bm, E)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print(f"B={Bn} T={T} r={r} n={n}: {dt*1e3:.2f} ms  {Bn*T/dt:.3e} traj-steps/s", flush=True)
