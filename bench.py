#!/usr/bin/env python3
"""Throughput benchmark of the fused EKS hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[3], "config 4"): a batch of 1024 videos x 17
keypoints, 5 ensemble members, 10 000 frames, single-view EKS -- 17 408
independent keypoint trajectories, 1.74e8 keypoint-timesteps per pass.  The
batch is fixed and sharded over the N ranks by video (strong scaling); at
N = 1 one GPU smooths all of it (7 GB of float32 member predictions).

A step = one pass of the hot path over the rank's shard, inputs resident in
HBM: ensemble median/variance over the 5 members -> forward Kalman filter ->
RTS backward pass -> projection + offsets, float64 recursions, smoothed
(x, y) float64 written to HBM (eks_smooth, include/eks_hip.h).  The model of
each trajectory (offsets, S0, Q from the low-variance
frames) is fitted once before timing (eks_amd.fit.singleview_model_batch)
and is not part of the step.

Synthetic data: per video a seeded (4 + video index)
Gaussian random walk per keypoint (sigma 2 px, start U(50, 450)), member
noise sigma_e ~ U(0.5, 3) px, 1 % outliers of 30 px; values float32.

Prints ONE JSON line (rank 0) with the throughput, the roofline of the
dominant kernel (HIP events on the launch stream) and the CPU baseline
(the numpy oracle on a bounded sample, 1 core).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "keypoint-timesteps smoothed/sec at 1/2/4/8 MI355X; max|Δ| vs CPU"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--videos", type=int, default=1024)
    ap.add_argument("--keypoints", type=int, default=17)
    ap.add_argument("--members", type=int, default=5)
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--smooth-param", type=float, default=0.01)
    ap.add_argument("--quantile-keep", type=float, default=25.0)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--algo", type=int, default=0, help="eks_smooth algo (0 auto)")
    ap.add_argument("--cpu-sample", type=int, default=24,
                    help="trajectories of the workload timed on the CPU oracle (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="after timing, gather all outputs to rank 0 once (RCCL) and report it")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: the video batch is split over ranks; weak: every rank "
                         "smooths --videos videos")
    return ap.parse_args()


def gen_videos(torch, videos, K, E, T, seed0, device):
    """(T, E, 2, B) float32 member predictions for the given video ids,
    trajectory index b = video_local * K + keypoint (innermost axis)."""
    B = len(videos) * K
    obs = torch.empty((T, E, 2, B), dtype=torch.float32, device=device)
    for i, v in enumerate(videos):
        g = torch.Generator(device=device)
        g.manual_seed(seed0 + v)
        f64 = dict(dtype=torch.float64, device=device, generator=g)
        start = torch.rand((1, 2, K), **f64) * 400.0 + 50.0
        steps = torch.randn((T, 2, K), **f64) * 2.0
        steps[0] = 0.0
        latent = start + torch.cumsum(steps, dim=0)                     # (T, 2, K)
        sig = torch.rand((1, E, 1, K), **f64) * 2.5 + 0.5
        x = latent[:, None] + torch.randn((T, E, 2, K), **f64) * sig
        out_mask = torch.rand((T, E, 1, K), **f64) < 0.01
        ang = torch.rand((T, E, 1, K), **f64) * (2 * math.pi)
        disp = torch.cat([torch.cos(ang), torch.sin(ang)], dim=2) * 30.0
        x = x + out_mask * disp
        obs[:, :, :, i * K:(i + 1) * K] = x.to(torch.float32)
    return obs


def fit_models(torch, lib_mod, obs_view, s, q, chunk=2048):
    """Per-trajectory single-view models, fitted on device in chunks."""
    from eks_amd import _lib, batch, fit
    B, T, E, n = obs_view.shape
    lib = _lib.load()
    parts = []
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        sub = obs_view[lo:hi]
        preds = torch.empty((hi - lo, T, n), dtype=torch.float64, device=obs_view.device)
        var = torch.empty_like(preds)
        sb, st, se, sj = sub.stride()
        _lib.check(lib.eks_ensemble(sub.data_ptr(), _lib.EKS_F32, hi - lo, T, E, n, sb, st, se,
                                    sj, _lib.EKS_MEDIAN, preds.data_ptr(), var.data_ptr(),
                                    _lib.stream_ptr()), "eks_ensemble")
        m = fit.singleview_model_batch(preds, var, s, q)
        parts.append(batch.pack_params(m["m0"], m["S0"], m["A"], m["Q"], m["C"], m["offset"],
                                       device=obs_view.device))
        del preds, var, m
    return torch.cat(parts, dim=0).contiguous()


def cpu_baseline(torch, obs_tm, out_view, n_traj, T, s, q):
    """Time the numpy oracle (the reference's algorithm, 1 core) on the first
    n_traj trajectories of the workload; compare with the GPU outputs."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    from oracle import eks_oracle as O
    idx = list(range(n_traj))
    host = obs_tm[:, :, :, :n_traj].cpu().numpy().astype(np.float64)  # (T, E, 2, b)
    gpu = out_view[:n_traj].cpu().numpy()
    maxdiff = 0.0
    with threadpool_limits(1):
        t0 = time.perf_counter()
        outs = []
        for b in idx:
            st = np.ascontiguousarray(np.transpose(host[..., b], (1, 0, 2)))  # (E, T, 2)
            out, _, _ = O.singleview_smooth(st, s, q)
            outs.append(out)
        dt = time.perf_counter() - t0
    for b, out in zip(idx, outs):
        maxdiff = max(maxdiff, float(np.abs(out - gpu[b]).max()))
    return dict(value=n_traj * T / dt, unit="kp-ts/s", cores=1, kind="port",
                sample=f"{n_traj} trajectories x {T} frames of this workload "
                       f"(oracle/eks_oracle.singleview_smooth: ensemble + fit + filter + "
                       f"smoother, numpy 1 thread), {dt:.1f} s"), maxdiff


def load_pmc(workload_key):
    path = os.path.join(HERE, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
    except Exception:
        return None
    if d.get("workload_key") != workload_key:
        return None
    return d


def main():
    a = parse()
    import torch
    from eks_amd import _lib, batch, dist
    rank, world, local = dist.init()
    if world != a.gpus and rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using {world}",
              file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    _lib.require_gpu()
    K, E, T = a.keypoints, a.members, a.frames
    if a.scaling == "strong":
        lo, hi = dist.shard_range(a.videos, world, rank)
    else:
        lo, hi = rank * a.videos, (rank + 1) * a.videos
    videos = range(lo, hi)
    B = len(videos) * K
    t_setup = time.perf_counter()
    obs_tm = gen_videos(torch, videos, K, E, T, a.seed, dev)          # (T, E, 2, B)
    obs = obs_tm.permute(3, 0, 1, 2)                                   # (B, T, E, 2) view
    params = fit_models(torch, _lib, obs, a.smooth_param, a.quantile_keep)
    out = torch.empty((T, B, 2), dtype=torch.float64, device=dev).permute(1, 0, 2)
    status = torch.empty((B,), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY  # single-view: A = C = I2

    def step():
        batch.smooth(obs, params, n=2, r=2, out=out, status=status, algo=a.algo, flags=flags)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if int((status != 0).sum().item()) != 0:
        raise RuntimeError("singular trajectories in the bench workload")
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = dist.max_over_ranks(elapsed, device=dev)
    # per-kernel launch durations: HIP events recorded by libeks_hip on the
    # launch stream between the kernels of each eks_smooth call (separate pass
    # so the events do not perturb the timed loop above)
    _lib.profile_begin(a.steps)
    for k in range(a.steps):
        step()
    kernels = _lib.profile_end()
    kern_ms = sum(ms for _, ms in kernels)
    kern_ms_max = dist.max_over_ranks(kern_ms, device=dev)
    units_local = B * T
    units_total = dist.sum_over_ranks(units_local, device=dev)

    gather_ms = None
    if a.gather and world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        local = out.permute(1, 0, 2).reshape(T, len(videos), K, 2).permute(1, 0, 2, 3)
        full = dist.gather_to_rank0(local.contiguous(), a.videos)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3
        del full

    cpu = None
    maxdiff = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.cpu_sample > 0:
        cpu, maxdiff = cpu_baseline(torch, obs_tm, out, min(a.cpu_sample, B), T,
                                    a.smooth_param, a.quantile_keep)

    if rank == 0:
        value = units_total / elapsed_max * a.steps
        bytes_per_unit = E * 2 * 4 + 2 * 8  # f32 members in, f64 (x, y) out
        achieved = bytes_per_unit * units_local / (kern_ms_max * 1e-3) / 1e9
        wk = f"config4-singleview-v{a.videos}-k{K}-e{E}-t{T}-n{world}-{a.scaling}"
        pmc = load_pmc(wk)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "kp-ts/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed_max / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"config 4: batch of {a.videos} videos x {K} keypoints x {E} "
                            f"members x {T} frames, single-view EKS (ensemble median/var -> "
                            f"forward KF -> RTS -> projection), float32 members, float64 "
                            f"recursions/outputs, {'split over' if a.scaling == 'strong' else 'per'} "
                            f"{world} GPU(s)",
                "videos": a.videos, "keypoints": K, "members": E, "frames": T,
                "trajectories_per_rank": B, "smooth_param": a.smooth_param,
                "quantile_keep": a.quantile_keep, "algo": a.algo,
                "parallelism": f"videos sharded over {world} rank(s), no data-path collective",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS,
                "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
                "kernel": "eks_smooth (" + " + ".join(n for n, _ in kernels) + ")",
                "kernel_ms": kern_ms_max,
                "kernels_ms": {n: round(ms, 4) for n, ms in kernels},
                "bytes_per_unit": bytes_per_unit,
                "units_per_launch": units_local,
            },
            "cpu_baseline": cpu,
            "max_abs_diff_vs_cpu": maxdiff,
            "setup_s": round(setup_s, 2),
        }
        if gather_ms is not None:
            line["gather_ms"] = gather_ms
        print(json.dumps(line))
    dist.barrier()


if __name__ == "__main__":
    main()
