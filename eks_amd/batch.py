"""Batched, device-resident API of the fused smoother (the throughput path).

    out = smooth(obs, params, n=..., r=...)

``obs`` is a CUDA tensor viewed as (B, T, E, n) -- B trajectories (video x
keypoint), T frames, E ensemble members, n observed coordinates -- float32 or
float64, ANY strides (the kernel reads obs[b*sb + t*st + e*se + j*sj]).
For coalesced loads give it a layout whose trajectory axis is innermost, e.g.
a contiguous (T, E, n, B) buffer viewed with ``.permute(3, 0, 1, 2)``:
that is what ``bench.py`` and ``make_time_major`` use.

``params`` is the (B, P) float64 tensor from ``pack_params``.  Nothing is
copied to the host; everything is stream-ordered on the current stream.
"""
from __future__ import annotations

import numpy as np

from . import _lib

_WS = {}


class Yev:
    """Ensemble hand-off planes (y, ev) written by ``fit(..., keep_yev=True)``
    and accepted by ``smooth`` in place of the member predictions (the
    members are then read once for fit + smooth; include/eks_hip.h
    eks_yev_bytes).  ``buf`` is a uint8 CUDA tensor; ``code`` the EKS_YEV32 /
    EKS_YEV64 input code."""

    def __init__(self, buf, B: int, T: int, E: int, n: int, code: int, mode: str):
        self.buf, self.B, self.T, self.E, self.n, self.code, self.mode = buf, B, T, E, n, code, mode
        self.shape = (B, T, E, n)
        self.device = buf.device


def param_len(n: int, r: int) -> int:
    return r + 3 * r * r + n * r + n


def pack_params(m0, S0, A, Q, C, offset, device="cuda"):  # noqa: C901
    """Pack per-trajectory models into the (B, P) layout of eks_param_len:
    [m0 (r) | S0 (r*r) | A (r*r) | Q (r*r) | C (n*r) | offset (n)].
    Inputs are arrays/tensors with a leading B axis (or none, = shared)."""
    import torch

    def t(x):
        x = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x,
                            dtype=torch.float64)
        return x

    m0, S0, A, Q, C, offset = map(t, (m0, S0, A, Q, C, offset))
    r = m0.shape[-1]
    n = offset.shape[-1]
    parts = [m0, S0, A, Q, C, offset]
    B = max(p.shape[0] if p.dim() == d else 1 for p, d in zip(parts, (2, 3, 3, 3, 3, 2)))
    flat = []
    for p, d in zip(parts, (2, 3, 3, 3, 3, 2)):
        if p.dim() == d - 1:
            p = p.unsqueeze(0).expand(B, *p.shape)
        flat.append(p.reshape(B, -1))
    out = torch.cat(flat, dim=1).contiguous().to(device)
    assert out.shape[1] == param_len(n, r)
    return out


def workspace(nbytes: int, device=None, slot: str = "smooth"):
    """Cached device scratch buffer per (device, slot); reused by later calls
    on the same stream (the kernels are stream-ordered)."""
    import torch
    dev = torch.device("cuda") if device is None else torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), slot)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        _WS[key] = buf
    return buf


# the pupil measurement matrix (eks/pupil_smoother.py:150-153; fit.PUPIL_C)
_PUPIL_C = np.array([[0, 1, 0], [-.5, 0, 1], [0, 1, 0], [.5, 0, 1],
                     [.5, 1, 0], [0, 0, 1], [-.5, 1, 0], [0, 0, 1]], dtype=np.float64)


def _diagonal(M) -> bool:
    off = ~np.eye(M.shape[-1], dtype=bool)
    return bool(np.all(M[..., off] == 0))


def model_flags(A, C, Q=None) -> int:
    """EKS_MODEL_* promise bits for host-side model arrays (A (.., r, r),
    C (.., n, r), Q (.., r, r)): A / C identity for every trajectory, or
    (with Q) the pupil structure -- C the pupil matrix, A and Q diagonal."""
    A = np.asarray(A)
    C = np.asarray(C)
    f = 0
    if A.shape[-1] == A.shape[-2] and np.all(A == np.eye(A.shape[-1])):
        f |= _lib.EKS_MODEL_A_IDENTITY
    if C.shape[-1] == C.shape[-2] and np.all(C == np.eye(C.shape[-1])):
        f |= _lib.EKS_MODEL_C_IDENTITY
    if (Q is not None and C.shape[-2:] == (8, 3) and np.all(C == _PUPIL_C)
            and _diagonal(A) and _diagonal(np.asarray(Q))):
        f |= _lib.EKS_MODEL_PUPIL
    return f


def smooth(obs, params, *, n: int, r: int, mode: str = "median", out=None, want_ms=False,
           want_nll=False, status=None, algo: int = 0, flags: int = 0, stream=None,
           check: bool = False, want_out: bool = True):
    """Fused ensemble -> forward -> backward -> projection for B trajectories.

    Returns dict(out=(B,T,n) view, ms=(B,T,r) or None, nll=(B,) or None,
    status=(B,) int32 bit mask).  ``out`` (if given) must be a (B, T, n)
    float64 CUDA tensor/view; by default a time-major buffer is allocated so
    that the kernel's stores are coalesced.  ``flags`` are EKS_MODEL_* promises
    (see ``model_flags``); ``algo`` 0 = automatic, 1 = sequential, 2 =
    time-parallel (three passes), 3 = time-parallel in two passes over the
    members, 4 = the runtime-n sequential kernel that every (r, n) without
    compiled kernels runs (include/eks_hip.h).  With ``check=True`` the call synchronises, raises on
    singular / mis-flagged trajectories and transparently re-runs with the
    sequential algorithm if the time-parallel scan reported a breakdown.
    """
    torch = _lib.require_gpu()
    if isinstance(obs, Yev):
        B, T, E, nn = obs.shape
        if nn != n:
            raise ValueError(f"obs has {nn} coordinates, expected n={n}")
        if mode != obs.mode:
            raise ValueError("the hand-off planes were made in another averaging mode")
        dt = obs.code
    else:
        if obs.dim() != 4:
            raise ValueError("obs must be viewed as (B, T, E, n)")
        B, T, E, nn = obs.shape
        if nn != n:
            raise ValueError(f"obs has {nn} coordinates, expected n={n}")
        if obs.dtype == torch.float32:
            dt = _lib.EKS_F32
        elif obs.dtype == torch.float64:
            dt = _lib.EKS_F64
        else:
            raise TypeError("obs must be float32 or float64")
    if mode not in ("median", "mean"):
        raise ValueError(f"{mode} averaging not supported")
    if params.shape != (B, param_len(n, r)) or params.dtype != torch.float64 \
            or not params.is_contiguous():
        raise ValueError(f"params must be a contiguous ({B}, {param_len(n, r)}) float64 tensor")
    dev = obs.device
    if not want_out:  # filter only: NLL per trajectory, no backward pass
        want_nll, want_ms, out = True, False, None
    elif out is None:
        out = torch.empty((T, B, n), dtype=torch.float64, device=dev).permute(1, 0, 2)
    ms = torch.empty((B, T, r), dtype=torch.float64, device=dev) if want_ms else None
    nll = torch.empty((B,), dtype=torch.float64, device=dev) if want_nll else None
    if status is None:
        status = torch.empty((B,), dtype=torch.int32, device=dev)
    lib = _lib.load()
    nbytes = lib.eks_smooth_workspace_bytes(B, T, n, r, E, algo)
    ws = workspace(nbytes, dev)
    sb, st, se, sj = (0, 0, 0, 0) if isinstance(obs, Yev) else obs.stride()
    ob, ot, oj = out.stride() if out is not None else (0, 0, 0)
    _lib.check(lib.eks_smooth(
        obs.buf.data_ptr() if isinstance(obs, Yev) else obs.data_ptr(), dt, B, T, E, n, r, sb, st, se, sj,
        _lib.EKS_MEDIAN if mode == "median" else _lib.EKS_MEAN, params.data_ptr(),
        out.data_ptr() if out is not None else None, ob, ot, oj,
        ms.data_ptr() if ms is not None else None,
        nll.data_ptr() if nll is not None else None, ws.data_ptr(), ws.numel(), flags, algo,
        status.data_ptr(), _lib.stream_ptr(stream)), "eks_smooth")
    res = dict(out=out, ms=ms, nll=nll, status=status)
    if check:
        st_all = status_bits(status)
        if st_all & _lib.EKS_STATUS_BAD_MODEL:
            raise ValueError("a model_flags promise (A = I / C = I / pupil structure) does not hold")
        if st_all & _lib.EKS_STATUS_SCAN and algo != 1:
            return smooth(obs, params, n=n, r=r, mode=mode, out=out, want_ms=want_ms,
                          want_nll=want_nll, status=status, algo=1, flags=flags,
                          stream=stream, check=True, want_out=want_out)
        if st_all & _lib.EKS_STATUS_SINGULAR:
            raise np.linalg.LinAlgError("Singular matrix")
    return res


def fit(obs, *, kind: str, n: int, r: int, smooth_param: float, quantile_keep: float,
        mode: str = "median", check: bool = True, params=None, status=None, keep_yev=False):
    """Batched model fit on the device (eks_fit, F2): (B, T, E, n) member view
    -> (B, eks_param_len(n, r)) float64 parameter rows for ``smooth``.

    kind "singleview" (r == n) or "multicam" (PCA with r
    axes; eks/multiview_pca_smoother.py:684-731)."""
    torch = _lib.require_gpu()
    if obs.dim() != 4 or obs.shape[3] != n:
        raise ValueError("obs must be viewed as (B, T, E, n)")
    B, T, E, _ = obs.shape
    dt = _lib.EKS_F32 if obs.dtype == torch.float32 else _lib.EKS_F64
    if obs.dtype not in (torch.float32, torch.float64):
        raise TypeError("obs must be float32 or float64")
    if mode not in ("median", "mean"):
        raise ValueError(f"{mode} averaging not supported")
    k = {"singleview": _lib.EKS_FIT_SINGLEVIEW, "multicam": _lib.EKS_FIT_MULTICAM}[kind]
    lib = _lib.load()
    if params is None:
        params = torch.empty((B, param_len(n, r)), dtype=torch.float64, device=obs.device)
    elif params.shape != (B, param_len(n, r)) or params.dtype != torch.float64 \
            or not params.is_contiguous():
        raise ValueError(f"params must be a contiguous ({B}, {param_len(n, r)}) float64 tensor")
    if status is None:
        status = torch.empty((B,), dtype=torch.int32, device=obs.device)
    ws = workspace(lib.eks_fit_workspace_bytes(B, T, n), obs.device, slot="fit")
    sb, st, se, sj = obs.stride()
    m = _lib.EKS_MEDIAN if mode == "median" else _lib.EKS_MEAN
    yev = None
    if keep_yev:
        # a Yev object (reused when passed in) receives the ensemble planes
        nbytes = lib.eks_yev_bytes(B, T, n, dt, E, m)
        if isinstance(keep_yev, Yev) and keep_yev.buf.numel() >= nbytes:
            yev = keep_yev
        else:
            yev = Yev(torch.empty(nbytes, dtype=torch.uint8, device=obs.device), B, T, E, n,
                      lib.eks_yev_dtype(dt, E, m), mode)
    _lib.check(lib.eks_fit(obs.data_ptr(), dt, B, T, E, n, r, sb, st, se, sj, m, k,
                           float(smooth_param), float(quantile_keep), params.data_ptr(),
                           ws.data_ptr(), ws.numel(), status.data_ptr(),
                           yev.buf.data_ptr() if yev is not None else None, _lib.stream_ptr()),
               "eks_fit")
    if check and bool((status != 0).any()):
        raise ValueError("eks_fit: no frame passed the variance threshold (NaN ensemble "
                         "variances?)")
    if keep_yev:
        return params, status, yev
    return params, status


def nll(obs, params, *, n: int, r: int, mode: str = "median", flags: int = 0, algo: int = 0,
        check: bool = True, status=None):
    """Filter-only pass: the innovation NLL of every
    trajectory / candidate model, no backward pass.  To score C candidate
    models of ONE trajectory, pass ``obs.expand(C, -1, -1, -1)`` (batch
    stride 0: the members are read once per candidate from the same memory)
    and C rows of params.  ``status`` (B,) int32 receives the per-trajectory
    status bits (check=False callers read it themselves)."""
    return smooth(obs, params, n=n, r=r, mode=mode, flags=flags, algo=algo, check=check,
                  want_out=False, status=status)["nll"]


def status_bits(status) -> int:
    """OR of all per-trajectory status words (synchronises)."""
    v = 0
    for bit in (_lib.EKS_STATUS_SINGULAR, _lib.EKS_STATUS_BAD_MODEL, _lib.EKS_STATUS_SCAN):
        if bool(((status & bit) != 0).any().item()):
            v |= bit
    return v


def make_time_major(stack_np, device="cuda", dtype=None):
    """(B, E, T, n) numpy array -> CUDA tensor stored (T, E, n, B), returned as
    the (B, T, E, n) view the kernels read with coalesced per-lane loads."""
    import torch
    a = np.asarray(stack_np)
    if dtype is not None:
        a = a.astype(dtype)
    tm = np.ascontiguousarray(np.transpose(a, (2, 1, 3, 0)))  # (T, E, n, B)
    d = torch.from_numpy(tm).to(device)
    return d.permute(3, 0, 1, 2)
