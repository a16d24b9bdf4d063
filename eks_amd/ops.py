"""``torch.ops.eks.*``: the C ABI entry points as PyTorch custom operators
("the torch extension wraps the same functions").

    import eks_amd.ops                       # registers the operators
    preds, vars_ = torch.ops.eks.ensemble(obs, "median")
    out, status = torch.ops.eks.smooth(obs, params, 2, 2, "median", 0, 0)

Each operator calls libeks_hip.so through ``eks_amd.batch`` / the ctypes table
(no CPU implementation: a CPU tensor raises), returns fresh contiguous
tensors, and has a fake (meta) implementation, so shapes propagate through
``torch.compile`` / FakeTensor tracing.  Layout conventions are those of
``eks_amd.batch``: obs is (B, T, E, n) with any strides.
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib, batch

_MODES = ("median", "mean")


def _need_cuda(*ts):
    for t in ts:
        if t.device.type != "cuda":
            raise RuntimeError("eks ops run on the GPU only (no CPU fallback): got a "
                               f"{t.device.type} tensor")


@torch.library.custom_op("eks::ensemble", mutates_args=())
def ensemble(obs: torch.Tensor, mode: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """(B, T, E, n) members -> (preds, vars) (B, T, n) float64
    (eks/ensemble_kalman.py:4-57, eks_ensemble)."""
    _need_cuda(obs)
    if mode not in _MODES:
        raise ValueError(f"{mode} averaging not supported")
    B, T, E, n = obs.shape
    preds = torch.empty((B, T, n), dtype=torch.float64, device=obs.device)
    var = torch.empty_like(preds)
    sb, st, se, sj = obs.stride()
    dt = _lib.EKS_F32 if obs.dtype == torch.float32 else _lib.EKS_F64
    _lib.check(_lib.load().eks_ensemble(obs.data_ptr(), dt, B, T, E, n, sb, st, se, sj,
                                        _lib.EKS_MEDIAN if mode == "median" else _lib.EKS_MEAN,
                                        preds.data_ptr(), var.data_ptr(), _lib.stream_ptr()),
               "eks_ensemble")
    return preds, var


@ensemble.register_fake
def _(obs, mode):
    B, T, E, n = obs.shape
    p = obs.new_empty((B, T, n), dtype=torch.float64)
    return p, torch.empty_like(p)


@torch.library.custom_op("eks::smooth", mutates_args=())
def smooth(obs: torch.Tensor, params: torch.Tensor, n: int, r: int, mode: str, flags: int,
           algo: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused ensemble -> forward -> backward -> projection (eks_smooth):
    (out (B, T, n) float64, status (B,) int32)."""
    _need_cuda(obs, params)
    res = batch.smooth(obs, params.contiguous(), n=n, r=r, mode=mode, flags=flags, algo=algo)
    return res["out"].contiguous(), res["status"].clone()


@smooth.register_fake
def _(obs, params, n, r, mode, flags, algo):
    B, T = obs.shape[0], obs.shape[1]
    return (obs.new_empty((B, T, n), dtype=torch.float64),
            obs.new_empty((B,), dtype=torch.int32))


@torch.library.custom_op("eks::nll", mutates_args=())
def nll(obs: torch.Tensor, params: torch.Tensor, n: int, r: int, mode: str,
        flags: int) -> torch.Tensor:
    """Filter-only innovation NLL per trajectory (eks_smooth with out = NULL)."""
    _need_cuda(obs, params)
    return batch.nll(obs, params.contiguous(), n=n, r=r, mode=mode, flags=flags).clone()


@nll.register_fake
def _(obs, params, n, r, mode, flags):
    return obs.new_empty((obs.shape[0],), dtype=torch.float64)


@torch.library.custom_op("eks::fit", mutates_args=())
def fit(obs: torch.Tensor, kind: str, n: int, r: int, smooth_param: float,
        quantile_keep: float, mode: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """Batched model fit (eks_fit): (params (B, P) float64, status (B,) int32)."""
    _need_cuda(obs)
    params, status = batch.fit(obs, kind=kind, n=n, r=r, smooth_param=smooth_param,
                               quantile_keep=quantile_keep, mode=mode, check=False)
    return params, status.clone()


@fit.register_fake
def _(obs, kind, n, r, smooth_param, quantile_keep, mode):
    B = obs.shape[0]
    return (obs.new_empty((B, batch.param_len(n, r)), dtype=torch.float64),
            obs.new_empty((B,), dtype=torch.int32))


@torch.library.custom_op("eks::newton_filter", mutates_args=())
def newton_filter(y: torch.Tensor, ev: torch.Tensor, mu0: torch.Tensor, S0: torch.Tensor,
                  A: torch.Tensor, Bm: torch.Tensor, E: torch.Tensor,
                  max_iter: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Newton "opti" forward filter (eks_newton_filter): (q (B, T, r), status)."""
    _need_cuda(y, ev)
    from .newton_eks import newton_filter_batch
    q, status = newton_filter_batch(y, ev, mu0, S0, A, Bm, E, max_iter)
    return q, status.clone()


@newton_filter.register_fake
def _(y, ev, mu0, S0, A, Bm, E, max_iter):
    B, T = y.shape[0], y.shape[1]
    r = mu0.shape[-1]
    return (y.new_empty((B, T, r), dtype=torch.float64),
            y.new_empty((B,), dtype=torch.int32))


@torch.library.custom_op("eks::interp1d", mutates_args=())
def interp1d(x: torch.Tensor, y: torch.Tensor, xq: torch.Tensor) -> torch.Tensor:
    """np.interp of every column of y (n, C) at xq (eks_interp1d), bit-identical."""
    _need_cuda(x, y, xq)
    from .smoothers import interp1d_linear
    return interp1d_linear(x, y, xq)


@interp1d.register_fake
def _(x, y, xq):
    return y.new_empty((xq.shape[0], y.shape[1]), dtype=torch.float64)


OPS = ("ensemble", "smooth", "nll", "fit", "newton_filter", "interp1d")
