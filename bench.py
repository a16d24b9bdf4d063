#!/usr/bin/env python3
"""Throughput benchmark of the fused EKS hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Default workload (BASELINE.json configs[3], "config 4"): a batch of 1024
videos x 17 keypoints, 5 ensemble members, 10 000 frames, single-view EKS --
17 408 independent keypoint trajectories, 1.74e8 keypoint-timesteps per
pass.  The batch is fixed and sharded over the N ranks by video (strong
scaling, no data-path collective); at N = 1 one GPU smooths all of it (7 GB
of float32 member predictions).  --config 2 / 3 / 5 run the other GPU
configurations of BASELINE.json (one keypoint set per rank: replicas).

A step = one pass of the hot path over the rank's trajectories, inputs
resident in HBM: ensemble median/variance over the members -> forward Kalman
filter -> RTS backward pass -> projection + offsets, float64 recursions,
smoothed coordinates (float64) written to HBM (eks_smooth in
include/eks_hip.h).  Config 5's step also scores an 8x8 grid of
(diameter_s, com_s) pupil models by their innovation NLL (one filter-only
batched call) before smoothing the best one.  Per-trajectory models (offsets,
S0, Q: SURVEY.md §8 A6-A8) are fitted once before timing.

Synthetic data: seeded random walks / AR(1) latents, member
noise sigma_e ~ U(0.5, 3) px, 1 % outliers of 30 px (single/multi-view);
values float32.

Prints ONE JSON line (rank 0): throughput, the roofline of the smoother's
kernels (HIP events recorded by libeks_hip on the launch stream), the CPU
baseline (the numpy oracle on a bounded sample, 1 core) and max|d| between
the GPU and CPU outputs on that sample.
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
PEAK_FP64_TFS = 78.6   # MI355X FP64 vector peak (AMD spec: half the 157.3 TF/s FP32 vector rate)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, choices=[2, 3, 4, 5],
                    help="BASELINE.json configuration (1-based index)")
    ap.add_argument("--videos", type=int, default=1024, help="config 4: videos in the batch")
    ap.add_argument("--keypoints", type=int, default=17)
    ap.add_argument("--cameras", type=int, default=4,
                    help="config 3: cameras V (n = 2V; V > 4 runs the runtime-n kernels)")
    ap.add_argument("--members", type=int, default=5)
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per video (default: 10k / 100k / 50k / 1M for configs 4/2/3/5)")
    ap.add_argument("--smooth-param", type=float, default=0.01)
    ap.add_argument("--quantile-keep", type=float, default=25.0)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--algo", type=int, default=0, help="eks_smooth algo (0 auto)")
    ap.add_argument("--cpu-cores", type=int, default=None,
                    help="processes of the all-core CPU baseline (default: the affinity mask, "
                         "capped by OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true",
                    help="config 4, N > 1: skip the final gather of all outputs to rank 0 "
                         "(RCCL), timed once after the throughput loop")
    ap.add_argument("--dense-pupil", action="store_true",
                    help="config 5: run the pupil model through the dense r=3, n=8 kernels "
                         "instead of the EKS_MODEL_PUPIL ones (comparison runs)")
    ap.add_argument("--timeshard", action="store_true",
                    help="config 5: split the frames over the ranks (eks_amd.timeshard: two "
                         "all_gathers of per-segment aggregates) instead of replicas")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step eagerly instead of replaying a captured HIP graph")
    ap.add_argument("--a3-lb", type=int, default=0,
                    help="tuning: algo 3's backward look-back (EKS_DBG_A3_LB: 0 auto, 1 off, 2 on)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="config 4: strong = the video batch is split over ranks; weak = "
                         "every rank smooths --videos videos")
    a = ap.parse_args()
    a.frames = a.frames or {4: 10000, 2: 100000, 3: 50000, 5: 1000000}[a.config]
    a.seed = a.config if a.seed is None else a.seed
    return a


# ---------------------------------------------------------------------------
# synthetic data
# ---------------------------------------------------------------------------
def gen_videos(torch, videos, K, E, T, seed0, device):
    """(T, E, 2, B) float32 single-view member predictions for the given video
    ids (seed seed0 + video id), trajectory b = video_local * K + keypoint."""
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


def ensemble_dev(torch, obs_view, mode="median"):
    """(B, T, n) preds / vars of a (B, T, E, n) member view (eks_ensemble)."""
    from eks_amd import _lib
    B, T, E, n = obs_view.shape
    preds = torch.empty((B, T, n), dtype=torch.float64, device=obs_view.device)
    var = torch.empty_like(preds)
    sb, st, se, sj = obs_view.stride()
    dt = _lib.EKS_F32 if obs_view.dtype == torch.float32 else _lib.EKS_F64
    _lib.check(_lib.load().eks_ensemble(obs_view.data_ptr(), dt, B, T, E, n, sb, st, se, sj,
                                        _lib.EKS_MEDIAN if mode == "median" else _lib.EKS_MEAN,
                                        preds.data_ptr(), var.data_ptr(), _lib.stream_ptr()),
               "eks_ensemble")
    return preds, var


# ---------------------------------------------------------------------------
# CPU baseline: the numpy oracle (oracle/eks_oracle.py) on the host cores,
# 1 core and one process per core, BLAS single-threaded in every process
# ---------------------------------------------------------------------------
def cpu_cores() -> int:
    """Cores the all-core baseline uses: the affinity mask, capped by the
    box's CPU share (OMP_NUM_THREADS / EKS_CPU_CORES, read before this
    process pins its own BLAS to one thread)."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("EKS_CPU_CORES") or os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_cores_cap() -> str:
    """Why ``cores`` can be below ``host_cpus``: the box's CPU share."""
    n = len(os.sched_getaffinity(0))
    for var in ("EKS_CPU_CORES", "OMP_NUM_THREADS"):
        cap = os.environ.get(var)
        if cap and cap.isdigit() and 0 < int(cap) < n:
            return (f"{var}={cap}: this job's CPU share on the box (the affinity mask shows "
                    f"{n} host CPUs shared with other jobs)")
    return "the affinity mask"


def _cpu_model(O, task):
    """Untimed model fit of one task, from its own ensemble."""
    kind, stack, args = task
    if kind == "nll":           # the model is given (a sweep candidate)
        return args
    preds, ev = O.ensemble_array(stack)
    if kind == "pupil":         # eks/pupil_smoother.py:109-172 (no variances)
        return O.pupil_params(preds, *args)
    fit = {"singleview": O.singleview_params, "multicam": O.multicam_params}[kind]
    return fit(preds, ev, *args)


def _cpu_hot(O, task, p):
    """The GPU step's scope for one task on the CPU: ensemble ->
    filtering_pass -> smooth_backward -> projection (eks/ensemble_kalman.py:
    4-164), or ensemble -> innovation NLL for a sweep candidate."""
    import numpy as np
    kind, stack, _ = task
    preds, ev = O.ensemble_array(stack)
    y = preds - p["means"]
    if kind == "nll":
        return O.compute_nll(y, p["m0"], p["S0"], p["C"], p["A"], p["Q"], ev)
    mf, Vf, S = O.filtering_pass(y, p["m0"], p["S0"], p["C"], np.eye(y.shape[1]), p["A"],
                                 p["Q"], ev)
    ms, _, _ = O.smooth_backward(y, mf, Vf, S, p["A"])
    return ms @ p["C"].T + p["means"]


def _cpu_worker(conn, barrier):
    """One process of the all-core baseline: fit its tasks (untimed), wait
    for every process, then time the hot path over its tasks."""
    from oracle import eks_oracle as O
    tasks = conn.recv()
    models = [_cpu_model(O, t) for t in tasks]
    barrier.wait()
    t0 = time.perf_counter()
    outs = [_cpu_hot(O, t, p) for t, p in zip(tasks, models)]
    t1 = time.perf_counter()
    conn.send((t0, t1, outs))
    conn.close()


def cpu_all_cores(tasks, cores):
    """Tasks round-robin over ``cores`` spawned processes (one BLAS thread
    each).  Returns (wall seconds of the timed hot phase: first start to last
    end, outputs in task order)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    cores = max(1, min(cores, len(tasks)))
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS",
                                            "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    barrier = ctx.Barrier(cores)
    procs, conns = [], []
    try:
        for i in range(cores):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_cpu_worker, args=(child, barrier), daemon=True)
            p.start()
            parent.send(tasks[i::cores])
            procs.append(p)
            conns.append(parent)
        res = [c.recv() for c in conns]
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        for p in procs:
            p.join(timeout=60)
    wall = max(r[1] for r in res) - min(r[0] for r in res)
    outs = [None] * len(tasks)
    for i, r in enumerate(res):
        outs[i::cores] = r[2]
    return wall, outs


def cpu_one_core(tasks):
    """Tasks in this process with one BLAS thread: (fit seconds, hot seconds
    per task, outputs)."""
    from threadpoolctl import threadpool_limits
    from oracle import eks_oracle as O
    t_fit = 0.0
    t_hot, outs = [], []
    with threadpool_limits(1):
        for t in tasks:
            f0 = time.perf_counter()
            p = _cpu_model(O, t)
            f1 = time.perf_counter()
            outs.append(_cpu_hot(O, t, p))
            t_fit += f1 - f0
            t_hot.append(time.perf_counter() - f1)
    return t_fit, t_hot, outs


# ---------------------------------------------------------------------------
# workloads: each returns a dict with step(), units, bytes_per_unit, cpu()
# ---------------------------------------------------------------------------
def workload_singleview(torch, a, dev, rank, world, config):
    from eks_amd import _lib, batch, dist
    K, E, T = a.keypoints, a.members, a.frames
    if config == 4:
        if a.scaling == "strong":
            lo, hi = dist.shard_range(a.videos, world, rank)
        else:
            lo, hi = rank * a.videos, (rank + 1) * a.videos
        videos = range(lo, hi)
    else:  # config 2: one video of K keypoints per rank (replicas)
        videos = range(0, 1)
    B = len(videos) * K
    obs_tm = gen_videos(torch, videos, K, E, T, a.seed, dev)          # (T, E, 2, B)
    obs = obs_tm.permute(3, 0, 1, 2)                                   # (B, T, E, 2) view
    fit_status = torch.empty((B,), dtype=torch.int32, device=dev)
    fit_kw = dict(kind="singleview", n=2, r=2, smooth_param=a.smooth_param,
                  quantile_keep=a.quantile_keep, status=fit_status)
    params, _ = batch.fit(obs, **fit_kw)                               # eks_fit (F2)
    out = torch.empty((T, B, 2), dtype=torch.float64, device=dev).permute(1, 0, 2)
    status = torch.empty((B,), dtype=torch.int32, device=dev)
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY  # single-view: A = C = I2

    def step():
        batch.smooth(obs, params, n=2, r=2, out=out, status=status, algo=a.algo, flags=flags)

    yev = {}

    def fit_step():
        # the model fit writes the ensemble planes; the smoother reads them,
        # so the member predictions are read once for fit + smooth
        yev["y"] = batch.fit(obs, params=params, check=False, keep_yev=yev.get("y", True),
                             **fit_kw)[2]

    def e2e_smooth():
        batch.smooth(yev["y"], params, n=2, r=2, out=out, status=status, algo=a.algo, flags=flags)

    def cpu_plan(cores):
        import numpy as np
        n_all = min(B, max(2, cores * (8 if config == 4 else 1)))
        host = obs_tm[:, :, :, :n_all].cpu().numpy().astype(np.float64)  # (T, E, 2, b)
        gpu = out[:n_all].cpu().numpy()
        tasks = [("singleview", np.ascontiguousarray(np.transpose(host[..., b], (1, 0, 2))),
                  (a.smooth_param, a.quantile_keep)) for b in range(n_all)]
        n_one = min(n_all, 32 if config == 4 else 2)
        return dict(tasks=tasks, gpu={b: gpu[b] for b in range(n_all)},
                    units_all=n_all * T, one=list(range(n_one)), units_one=n_one * T,
                    what=f"{{n}} trajectories x {T} frames of this workload")

    desc = (f"config {config}: " + (f"batch of {a.videos} videos x " if config == 4 else "1 video x ")
            + f"{K} keypoints x {E} members x {T} frames, single-view EKS (ensemble median/var "
            f"-> forward KF -> RTS -> projection), float32 members, float64 recursions/outputs")
    return dict(step=step, fit_step=fit_step, e2e_smooth=e2e_smooth, status=status, units=B * T,
                bytes_per_unit=E * 2 * 4 + 2 * 8, cpu_plan=cpu_plan, desc=desc,
                cfg=dict(videos=a.videos if config == 4 else 1, keypoints=K, members=E, frames=T,
                         trajectories_per_rank=B, smooth_param=a.smooth_param,
                         quantile_keep=a.quantile_keep),
                shape=(B, T, 2, 2, E),
                # PMC traffic is a property of one rank's launch: keyed by the
                # rank's own shard (videos per rank), so an N-rank line finds
                # the profile of an N = 1 run of the same shard size
                key=f"config{config}-singleview-v{len(videos)}-k{K}-e{E}-t{T}",
                out=out, videos=videos)


def workload_multiview(torch, a, dev, rank, world):
    """config 3: V cameras (4 by default) x 17 keypoints x 50k frames, PCA multiview."""
    import numpy as np
    from eks_amd import _lib, batch, fit, synthetic
    K, E, T, V = a.keypoints, a.members, a.frames, a.cameras
    rng = np.random.default_rng(a.seed)
    st = synthetic.multiview_obs(rng, V, E, T, K=K)                   # (E, T, K, 8) f32
    n = 2 * V
    obs_tm = torch.from_numpy(np.ascontiguousarray(st.transpose(1, 0, 3, 2))).to(dev)  # (T,E,8,K)
    obs = obs_tm.permute(3, 0, 1, 2)
    fit_status = torch.empty((K,), dtype=torch.int32, device=dev)
    fit_kw = dict(kind="multicam", n=n, r=3, smooth_param=a.smooth_param,
                  quantile_keep=a.quantile_keep, status=fit_status)
    params, _ = batch.fit(obs, **fit_kw)                               # eks_fit (F2): PCA model
    flags = _lib.EKS_MODEL_A_IDENTITY                                  # A = I3 by construction
    out = torch.empty((T, K, n), dtype=torch.float64, device=dev).permute(1, 0, 2)
    status = torch.empty((K,), dtype=torch.int32, device=dev)

    def step():
        batch.smooth(obs, params, n=n, r=3, out=out, status=status, algo=a.algo, flags=flags)

    yev = {}

    def fit_step():
        yev["y"] = batch.fit(obs, params=params, check=False, keep_yev=yev.get("y", True),
                             **fit_kw)[2]

    def e2e_smooth():
        batch.smooth(yev["y"], params, n=n, r=3, out=out, status=status, algo=a.algo, flags=flags)

    def cpu_plan(cores):
        n_all = min(K, max(2, cores))
        gpu = out[:n_all].cpu().numpy()
        tasks = [("multicam", st[:, :, k, :].astype(np.float64), (a.smooth_param, a.quantile_keep))
                 for k in range(n_all)]
        return dict(tasks=tasks, gpu={k: gpu[k] for k in range(n_all)},
                    units_all=n_all * T, one=[0, 1], units_one=2 * T,
                    what=f"{{n}} keypoints x {T} frames x {V} cameras of this workload")

    desc = (f"config 3: multiview PCA smoother, {V} cameras x {K} keypoints x {E} members x "
            f"{T} frames (r=3 latent, n={n}), float32 members, float64 recursions/outputs")
    return dict(step=step, fit_step=fit_step, e2e_smooth=e2e_smooth, status=status,
                units=K * T, bytes_per_unit=E * n * 4 + n * 8, cpu_plan=cpu_plan, desc=desc,
                cfg=dict(cameras=V, keypoints=K, members=E, frames=T,
                         smooth_param=a.smooth_param, quantile_keep=a.quantile_keep),
                shape=(K, T, n, 3, E),
                key=f"config3-multiview-k{K}-e{E}-t{T}" + (f"-v{V}" if V != 4 else ""))


def workload_pupil(torch, a, dev, rank, world):
    """config 5: IBL pupil, 1M frames x 4 keypoints, NLL sweep + smooth."""
    import numpy as np
    from eks_amd import _lib, batch, fit, synthetic
    E, T = a.members, a.frames
    st = synthetic.pupil_obs(np.random.default_rng(a.seed), E, T, a=0.99)  # (E, T, 8) f32
    obs_tm = torch.from_numpy(np.ascontiguousarray(st.transpose(1, 0, 2))).to(dev)  # (T, E, 8)
    obs = obs_tm.unsqueeze(0)                                          # (1, T, E, 8) view
    preds, _ = ensemble_dev(torch, obs)
    preds = preds[0].cpu().numpy()
    d_grid = 1.0 - np.geomspace(1e-4, 1e-1, 8)
    c_grid = 1.0 - np.geomspace(1e-4, 1e-1, 8)
    base = fit.pupil_model(preds, np.diag([0.99, 0.99, 0.99]))
    var0 = np.diag(base["S0"])
    cands = []
    for d in d_grid:
        for c in c_grid:
            A = np.diag([d, c, c])
            cands.append(dict(base, A=A, Q=np.diag(var0 * (1 - np.diag(A) ** 2))))
    stackp = lambda key: np.stack([m[key] for m in cands])  # noqa: E731
    params = batch.pack_params(stackp("m0"), stackp("S0"), stackp("A"), stackp("Q"), stackp("C"),
                               stackp("offset"), device=dev)
    out = torch.empty((T, 1, 8), dtype=torch.float64, device=dev).permute(1, 0, 2)
    ms = torch.empty((1, T, 3), dtype=torch.float64, device=dev)
    status = torch.empty((1,), dtype=torch.int32, device=dev)
    sweep_status = torch.empty((len(cands),), dtype=torch.int32, device=dev)
    cands_obs = obs.expand(len(cands), -1, -1, -1)  # batch stride 0: members shared
    # pupil structure (C = pupil matrix, A / Q diagonal): EKS_MODEL_PUPIL kernels
    flags = 0 if a.dense_pupil else batch.model_flags(stackp("A"), stackp("C"), stackp("Q"))
    state = {}
    t0, Tk = 0, T
    if a.timeshard:
        from eks_amd import timeshard
        t0, Tk = timeshard.split_frames(T, world, rank)
        seg_out = out[:, t0:t0 + Tk]

    def step_timeshard():
        scores = timeshard.smooth_time_sharded(cands_obs[:, t0:t0 + Tk], params, n=8, r=3,
                                               t_base=t0, T_total=T, want_out=False,
                                               flags=flags)["nll"]
        best = torch.argmin(scores)            # the same on every rank (summed NLL)
        p_best = params.index_select(0, best.view(1)).contiguous()
        r = timeshard.smooth_time_sharded(obs[:, t0:t0 + Tk], p_best, n=8, r=3, t_base=t0,
                                          T_total=T, out=seg_out, want_ms=True, flags=flags)
        state["best"], state["scores"], state["ms"] = best, scores, r["ms"]
        status.copy_(r["status"])

    def step():
        scores = batch.nll(cands_obs, params, n=8, r=3, algo=a.algo, check=False, flags=flags,
                           status=sweep_status)
        best = torch.argmin(scores)                                    # stays on device
        p_best = params.index_select(0, best.view(1)).contiguous()
        r = batch.smooth(obs, p_best, n=8, r=3, out=out, want_ms=True, status=status,
                         algo=a.algo, flags=flags)
        state["best"], state["scores"], state["ms"] = best, scores, r["ms"]

    def cpu_plan(cores):
        # the step's scope on a bounded prefix of Tc frames: every candidate's
        # NLL (eks_amd batch.nll <-> oracle compute_nll) + smoothing the chosen one
        from oracle import eks_oracle as O
        Tc = min(T, 20000)
        pre = np.ascontiguousarray(st[:, :Tc].astype(np.float64))
        b = int(state["best"].item())
        tasks = [("nll", pre, dict(c, means=c["offset"])) for c in cands]
        tasks.append(("pupil", pre, (cands[b]["A"],)))
        # the GPU output for the same prefix and model
        pm = fit.pupil_model(O.ensemble_array(pre)[0], cands[b]["A"])
        pb = batch.pack_params(pm["m0"], pm["S0"], pm["A"], pm["Q"], pm["C"], pm["offset"],
                               device=dev)
        # the timed step's kernels (same model flags: the EKS_MODEL_PUPIL
        # kernels unless --dense-pupil) on the same prefix
        fb = 0 if a.dense_pupil else batch.model_flags(pm["A"][None], pm["C"][None], pm["Q"][None])
        g = batch.smooth(obs[:, :Tc], pb, n=8, r=3, flags=fb, check=True)["out"][0].cpu().numpy()
        # the sweep's scores on the same prefix, for the candidates the 1-core
        # run scores (tasks 0 and 1): relative NLL difference
        nll_gpu = batch.nll(cands_obs[:2, :Tc], params[:2].contiguous(), n=8, r=3, flags=flags,
                            check=True).cpu().numpy()
        half = len(cands) // 2
        return dict(tasks=tasks, gpu={len(cands): g}, units_all=4 * Tc, units_one=4 * Tc,
                    nll_gpu={0: float(nll_gpu[0]), 1: float(nll_gpu[1])},
                    one=[0, 1, len(cands)], weights=[half, half, 1],
                    what=f"first {Tc} frames x 4 keypoints: NLL of {{n}} of the {len(cands)} "
                         f"candidate models + smoothing the chosen one")

    desc = (f"config 5: IBL-pupil smoother, {T} frames x 4 keypoints x {E} members (r=3 latent, "
            f"n=8): NLL sweep over {len(cands)} (diameter_s, com_s) models (filter-only, "
            f"batched) + smoothing of the argmin, float64")
    if a.timeshard:
        desc += f"; frames split over {world} rank(s) (time-sharded scan)"
    def post_check():
        # after the timed loop: no scan breakdown / singular system in the
        # sweep (its NLLs feed the argmin unchecked) or in the final smooth
        bad = _lib.EKS_STATUS_SCAN | _lib.EKS_STATUS_SINGULAR
        if not a.timeshard and int((sweep_status & bad).sum().item()) != 0:
            raise RuntimeError("config 5: the NLL sweep reported a scan breakdown / singular system")
        if int((status & bad).sum().item()) != 0:
            raise RuntimeError("config 5: the final smooth reported a scan breakdown / singular system")

    return dict(step=step_timeshard if a.timeshard else step, status=status, units=4 * Tk,
                post_check=post_check,
                bytes_per_unit=(32 * E + 88) / 4, cpu_plan=cpu_plan, desc=desc,
                timeshard=a.timeshard,
                # k_c1_elem: one element-absorb step per (candidate, frame); flops counted
                # from kf_steps.hpp elem_absorb (FMA = 2): pupil kernels 27 (diagonal
                # predict) + 42 (two folded pairs) + 2 x 76 + 4 x 92 (sparse rows) = 589;
                # dense r = 3, n = 8: 162 + 8 x 123 = 1146
                flops=dict(kernel="k_c1_elem", per_unit=1146 if a.dense_pupil else 589,
                           units=(len(cands) + 1) * Tk,  # the sweep + the chosen model's smooth
                           unit_is="element-absorb step"),
                cfg=dict(frames=T, keypoints=4, members=E, candidates=len(cands)),
                shape=(1, T, 8, 3, E),
                key=f"config5-pupil-t{T}" + (f"-ts-n{world}" if a.timeshard else ""),
                extra=lambda: dict(
                    sweep_candidates=len(cands),
                    best_model=[float(x) for x in np.diag(cands[int(state['best'])]['A'])]))


def assert_clean(torch, w, where):
    """Raise if the step's last call flagged any trajectory (singular system,
    broken model promise, or a scan / chain-wait breakdown: EKS_STATUS_*),
    plus the workload's own checks.  Run after every loop over the step, so a
    timed loop never reports a number from a silently failed call."""
    from eks_amd import batch
    bad = int((w["status"] != 0).sum().item())
    if bad:
        raise RuntimeError(f"{where}: {bad} trajectories reported status bits "
                           f"(OR = {batch.status_bits(w['status'])}: 1 singular, 2 model "
                           "promise broken, 4 scan / chain-wait breakdown)")
    if "post_check" in w:
        w["post_check"]()


def load_pmc(workload_key, path=None):
    """PMC summary of one rank's launch of this workload (tools/gpu_profile.sh
    -> tools/prof_summary.py): bench_pmc.json holds one entry per workload
    key (per-rank shard), or None."""
    path = path or os.path.join(HERE, "bench_pmc.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
    except Exception:
        return None
    return (d.get("entries") or {}).get(workload_key)


def launch_ranks(a) -> int:
    """``--gpus N`` without a launcher: run N ranks of this script under
    torch.distributed.run as a child process (started before this process
    touches the GPU) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def runs_cpu_baseline(rank, a) -> bool:
    """The CPU baseline runs on rank 0's own shard after the timed loop, at
    any N (for N > 1 the other ranks wait at the final barrier)."""
    return rank == 0 and not a.no_cpu_baseline


def make_line(a, w, world, algo_used, units_local, units_total, elapsed_max, kernels,
              kern_ms_max, cpu, maxdiff, e2e, cpu_e2e, gather_ms, gather_bytes, setup_s,
              hip_graph, backend, pmc_path=None):
    """The one JSON line rank 0 prints (the driver's bench contract).  At N > 1
    the roofline, traffic and CPU baseline describe rank 0's own launch (its
    shard); ``value`` is the whole job's units over the max-over-ranks time."""
    value = units_total / elapsed_max * a.steps
    # the roofline's rate per launch: algorithmic bytes of the rank's launch
    # over the graph-replayed step time (max over ranks, the driver's clock);
    # the eager HIP-event kernel sum is reported beside it (it omits the
    # memset node and the launch gaps the replay pays)
    step_ms = elapsed_max / a.steps * 1e3
    achieved = w["bytes_per_unit"] * units_local / (step_ms * 1e-3) / 1e9
    achieved_ev = w["bytes_per_unit"] * units_local / (kern_ms_max * 1e-3) / 1e9
    pmc = load_pmc(w["key"], pmc_path)
    scaling = ("strong" if (a.config == 4 and a.scaling == "strong") or w.get("timeshard")
               else "weak")
    par = (f"videos sharded over {world} rank(s), no data-path collective" if a.config == 4
           else f"frames split over {world} rank(s), 2 all_gathers of segment aggregates"
           if w.get("timeshard") else f"{world} independent replica(s)")
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "kp-ts/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed_max / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": dict(workload=w["desc"], algo=algo_used, parallelism=par, **w["cfg"]),
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBS,
            "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
            "traffic_key": w["key"],
            "kernel": "eks_smooth (" + " + ".join(n for n, _ in kernels) + ")",
            "time_basis": "ms_per_step (graph replay)",
            "kernel_ms": kern_ms_max,
            "achieved_kernel_events": achieved_ev,
            "frac_kernel_events": achieved_ev / PEAK_HBM_GBS,
            "kernels_ms": {n: round(ms, 4) for n, ms in kernels},
            "bytes_per_unit": w["bytes_per_unit"],
            "units_per_launch": units_local,
        },
        "cpu_baseline": cpu,
        "max_abs_diff_vs_cpu": maxdiff,
        "end_to_end": None if e2e is None else dict(e2e, cpu_value=cpu_e2e),
        "setup_s": round(setup_s, 2),
        "hip_graph": hip_graph,
    }
    if "flops" in w:  # an FP64-issue-bound kernel: its flop roofline beside the HBM one
        f = w["flops"]
        kms = dict(kernels).get(f["kernel"])
        if kms:
            tf = f["per_unit"] * f["units"] / (kms * 1e-3) / 1e12
            line["flop_roofline"] = dict(kernel=f["kernel"], bound="fp64 valu", achieved=tf,
                                         peak=PEAK_FP64_TFS, unit="TFLOP/s",
                                         frac=tf / PEAK_FP64_TFS, flops_per_unit=f["per_unit"],
                                         units_per_launch=f["units"], unit_is=f["unit_is"])
    if "extra" in w:
        line.update(w["extra"]())
    if world > 1:
        line["distributed"] = dict(world_size=world, backend=backend, units_per_rank=units_local,
                                   roofline_scope="rank 0's launch (per-rank shard)")
    if gather_ms is not None:
        # config 4 is "sharded over N GPUs (RCCL gather)": the rate with the
        # one gather of every output to rank 0 priced in (once per job, not
        # per step: kp-ts over the step time plus the gather time)
        line["gather_ms"] = gather_ms
        line["gather_bytes"] = gather_bytes
        line["value_with_gather"] = units_total / (elapsed_max / a.steps + gather_ms * 1e-3)
    return line


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    import torch
    from eks_amd import _lib, dist
    from threadpoolctl import threadpool_limits
    rank, world, local = dist.init()
    if world != a.gpus and rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using {world}",
              file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    _lib.require_gpu()
    t_setup = time.perf_counter()
    if a.a3_lb:
        _lib.debug_set(_lib.EKS_DBG_A3_LB, a.a3_lb)
    if a.config in (2, 4):
        w = workload_singleview(torch, a, dev, rank, world, a.config)
    elif a.config == 3:
        w = workload_multiview(torch, a, dev, rank, world)
    else:
        w = workload_pupil(torch, a, dev, rank, world)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    step = w["step"]
    # the algorithm eks_smooth resolves for this shape (0 = automatic choice)
    algo_used = int(_lib.load().eks_smooth_algo(*w["shape"], a.algo))
    w["key"] += f"-a{algo_used}"

    tw = time.perf_counter()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # (a rough step time, only to size the pre-timing warm replays below)
    step_est = (time.perf_counter() - tw) / max(1, a.warmup)
    assert_clean(torch, w, "warm-up")
    # the step's kernel sequence captured once as a HIP graph (hipGraph via
    # torch.cuda.CUDAGraph: the C ABI launches on the capturing stream and
    # allocates nothing), replayed in the timed loop; eager launches if the
    # capture is refused
    graph = None
    # (a time-sharded step exchanges through host-side collectives: eager)
    if not a.no_graph and not (w.get("timeshard") and world > 1):
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            g.replay()
            torch.cuda.synchronize()
            graph = g
        except Exception as exc:  # pragma: no cover - depends on the runtime
            print(f"[bench] HIP graph capture failed ({exc}); launching eagerly",
                  file=sys.stderr)
    eager_step = step
    warm_replays = 0
    if graph is not None:
        step = graph.replay
        # the replays warmed right before the timed region as well: after the
        # capture's idle gap the GPU runs ~7-10 % slow for the next ~10 ms of
        # work (tools/first_step.py, profiles/r05/ab8), which W = 5 steps of
        # a small shard (0.5 ms each) do not cover: at least W replays and
        # at least ~30 ms of them (untimed; reported as warmup_replays)
        warm_replays = max(a.warmup, min(200, int(math.ceil(0.03 / max(step_est, 1e-5)))))
        for _ in range(warm_replays):
            step()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = dist.max_over_ranks(elapsed, device=dev)
    assert_clean(torch, w, "timed loop")
    # per-kernel launch durations: HIP events recorded by libeks_hip on the
    # launch stream around each kernel of each eks_smooth call (separate pass,
    # so the events do not perturb the timed loop above)
    _lib.profile_begin(8 * a.steps)
    for _ in range(a.steps):
        eager_step()
    kernels = [(n, ms / a.steps) for n, ms in _lib.profile_end()]  # per step
    assert_clean(torch, w, "kernel-timing loop")
    kern_ms = sum(ms for _, ms in kernels)
    kern_ms_max = dist.max_over_ranks(kern_ms, device=dev)
    units_local = w["units"]
    units_total = dist.sum_over_ranks(units_local, device=dev)

    # end to end: the model fit on the device (eks_fit) + the hot path, i.e.
    # what the reference's per-keypoint wrappers do from member predictions
    e2e = None
    if "fit_step" in w:
        fit_step, e2e_smooth = w["fit_step"], w["e2e_smooth"]

        def e2e_eager():
            fit_step()
            e2e_smooth()

        tw = time.perf_counter()
        for _ in range(max(1, a.warmup)):
            e2e_eager()
        torch.cuda.synchronize()
        e2e_est = (time.perf_counter() - tw) / max(1, a.warmup)
        # replayed as one HIP graph like the hot-path step (eager: ~15 launches
        # whose host cost the small configurations would otherwise time)
        e2e_run = e2e_eager
        if graph is not None:
            try:
                ge = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ge):
                    e2e_eager()
                ge.replay()
                torch.cuda.synchronize()
                e2e_run = ge.replay
                # (warm as the hot-path replays above: >= W and >= ~30 ms)
                for _ in range(max(a.warmup, min(200, int(math.ceil(0.03 / max(e2e_est, 1e-5)))))):
                    e2e_run()
            except Exception as exc:  # pragma: no cover - depends on the runtime
                print(f"[bench] end-to-end graph capture failed ({exc}); launching eagerly",
                      file=sys.stderr)
        dist.barrier()
        torch.cuda.synchronize()
        f0 = time.perf_counter()
        for _ in range(a.steps):
            e2e_run()
        torch.cuda.synchronize()
        dist.barrier()
        e2e_s = dist.max_over_ranks(time.perf_counter() - f0, device=dev)
        assert_clean(torch, w, "end-to-end loop")
        _lib.profile_begin(8 * a.steps)
        for _ in range(a.steps):
            fit_step()
            e2e_smooth()
        fit_kernels = [(n, ms / a.steps) for n, ms in _lib.profile_end()]
        assert_clean(torch, w, "end-to-end kernel-timing loop")
        e2e = dict(value=units_total / e2e_s * a.steps, ms_per_step=e2e_s / a.steps * 1e3,
                   hip_graph=e2e_run is not e2e_eager,
                   kernels_ms={n: round(ms, 4) for n, ms in fit_kernels},
                   scope="eks_fit (ensemble, good-frame percentile, model fit; writes the "
                         "ensemble planes) + eks_smooth from those planes (members read once)")

    # the one data-path collective of the batch job: every
    # rank's smoothed (videos, T, K, 2) float64 block gathered to rank 0 over
    # RCCL, timed once after the throughput loop, never inside ``value``
    gather_ms = None
    gather_bytes = None
    if not a.no_gather and world > 1 and a.config == 4:
        T, K = a.frames, a.keypoints
        nv = len(w["videos"])
        loc = w["out"].permute(1, 0, 2).reshape(T, nv, K, 2).permute(1, 0, 2, 3).contiguous()
        total_videos = nv * world if a.scaling == "weak" else a.videos
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        full = dist.gather_to_rank0(loc, total_videos)
        torch.cuda.synchronize()
        gather_ms = dist.max_over_ranks((time.perf_counter() - g0) * 1e3, device=dev)
        if rank == 0:
            gather_bytes = full.numel() * full.element_size()
            # rank 0's own block arrives unchanged
            assert torch.equal(full[:nv], loc), "gather: rank 0 block differs"
        del full

    cpu = None
    maxdiff = None
    nll_rel = None
    cpu_e2e = None
    if runs_cpu_baseline(rank, a):
        cores = cpu_cores() if a.cpu_cores is None else a.cpu_cores
        plan = w["cpu_plan"](cores)
        tasks = plan["tasks"]
        one = [tasks[i] for i in plan["one"]]
        t_fit1, hot1, outs1 = cpu_one_core(one)
        wts = plan.get("weights") or [1] * len(one)
        t_hot1 = sum(wi * ti for wi, ti in zip(wts, hot1))
        used = max(1, min(cores, len(tasks)))
        wall, outs = cpu_all_cores(tasks, used)
        diffs = [float(abs(outs[i] - g).max()) for i, g in plan["gpu"].items()]
        diffs += [float(abs(outs1[j] - plan["gpu"][i]).max())
                  for j, i in enumerate(plan["one"]) if i in plan["gpu"]]
        maxdiff = max(diffs)
        if plan.get("nll_gpu"):  # candidate NLLs: GPU sweep vs the oracle's compute_nll
            nll_rel = max(abs(outs1[j] - v) / abs(outs1[j]) for j, v in plan["nll_gpu"].items())
        if plan.get("weights") is None:
            cpu_e2e = plan["units_one"] / (t_fit1 + t_hot1)
        if plan.get("weights") is not None:
            one_desc = (plan["what"].format(n=len(one) - 1) + " (the candidates' time scaled "
                        f"x{plan['weights'][0]} to all of them)")
        else:
            one_desc = plan["what"].format(n=len(one))
        cpu = dict(value=plan["units_all"] / wall, unit="kp-ts/s", cores=used, kind="port",
                   value_1core=plan["units_one"] / t_hot1,
                   sample=(plan["what"].format(n=len(tasks) - (1 if plan.get("weights") else 0)) + f", {used} processes x 1 thread "
                           f"(numpy oracle: ensemble + filtering_pass + smooth_backward + "
                           f"projection; model fit untimed), {wall:.1f} s wall; 1-core figure "
                           f"on {one_desc}, {t_hot1:.1f} s"),
                   host_cpus=len(os.sched_getaffinity(0)),
                   cores_cap=cpu_cores_cap())

    if rank == 0:
        backend = None
        if world > 1:
            import torch.distributed as tdist
            backend = str(tdist.get_backend())
        line = make_line(a, w, world, algo_used, units_local, units_total, elapsed_max, kernels,
                         kern_ms_max, cpu, maxdiff, e2e, cpu_e2e, gather_ms, gather_bytes,
                         setup_s, graph is not None, backend)
        if nll_rel is not None:
            line["nll_rel_diff_vs_cpu"] = nll_rel
        line["warmup_replays"] = warm_replays
        print(json.dumps(line))
    dist.barrier()


if __name__ == "__main__":
    main()
