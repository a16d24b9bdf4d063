"""Drop-in replacements for the reference's core functions.

Same names, arguments, return values, dtypes, side effects and errors as
eks/ensemble_kalman.py (erialc-cal/eks):

    ensemble(markers_list, keys, mode='median')                 :4-57
    filtering_pass(y, m0, S0, C, R, A, Q, ensemble_vars)         :59-107
    kalman_dot(array, V, C, R)                                   :110-117
    smooth_backward(y, mf, Vf, S, A, Q, C)                       :120-164

plus the names BASELINE.json's north star uses for them in later upstream
versions (``forward_pass`` = filtering_pass, ``backward_pass`` =
smooth_backward) and ``compute_nll`` (the filter's Gaussian innovation
negative log-likelihood; SURVEY.md §8 A5 -- the reference has none).

numpy in, numpy out: arrays are moved to the GPU, the HIP kernels of
libeks_hip.so do the work, results come back as float64 numpy arrays.  A
singular innovation or smoother matrix raises ``numpy.linalg.LinAlgError``
(the reference's np.linalg.solve does); a bad ``mode`` raises ValueError.
For throughput on many trajectories use ``eks_amd.batch`` instead.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

from . import _lib


def _to_dev(a, torch, dtype=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64 if dtype is None else dtype))
    return torch.from_numpy(a).to("cuda")


def _raise_if_singular(status, what):
    if status is not None and bool((status != 0).any()):
        raise np.linalg.LinAlgError(f"Singular matrix ({what})")


# --------------------------------------------------------------------------
def ensemble_array(stack, mode: str = "median"):
    """(E, T, n) member array -> (preds (T, n), vars (T, n)) on the GPU."""
    torch = _lib.require_gpu()
    if mode == "median":
        m = _lib.EKS_MEDIAN
    elif mode == "mean":
        m = _lib.EKS_MEAN
    else:
        raise ValueError(f"{mode} averaging not supported")
    stack = np.asarray(stack, dtype=np.float64)
    E, T, n = stack.shape
    d = _to_dev(stack, torch)
    preds = torch.empty((T, n), dtype=torch.float64, device="cuda")
    var = torch.empty_like(preds)
    lib = _lib.load()
    _lib.check(lib.eks_ensemble(d.data_ptr(), _lib.EKS_F64, 1, T, E, n, 0, n, T * n, 1, m,
                                preds.data_ptr(), var.data_ptr(), _lib.stream_ptr()),
               "eks_ensemble")
    return preds.cpu().numpy(), var.cpu().numpy()


def ensemble_handoff(stack, mode: str = "median"):
    """(E, T, n) member array -> (yev, preds (T, n), vars (T, n)).

    Like ``ensemble_array``, but the device ensemble is written straight into
    the y / ev hand-off planes that ``batch.smooth`` accepts in place of the
    members (include/eks_hip.h eks_yev_bytes; for one trajectory the y and ev
    planes are the (T, n) arrays, ev starting at the next 256-byte boundary).
    The per-keypoint wrappers fit their model on the host copies and smooth
    from the planes: the members are uploaded and reduced once, not twice."""
    from .batch import Yev
    torch = _lib.require_gpu()
    if mode == "median":
        m = _lib.EKS_MEDIAN
    elif mode == "mean":
        m = _lib.EKS_MEAN
    else:
        raise ValueError(f"{mode} averaging not supported")
    stack = np.asarray(stack, dtype=np.float64)
    E, T, n = stack.shape
    d = _to_dev(stack, torch)
    lib = _lib.load()
    code = lib.eks_yev_dtype(_lib.EKS_F64, E, m)
    if code != _lib.EKS_YEV64:
        raise RuntimeError(f"eks_yev_dtype(F64) = {code}, expected EKS_YEV64")
    nbytes = lib.eks_yev_bytes(1, T, n, _lib.EKS_F64, E, m)
    ev_off = (T * n * 8 + 255) // 256 * 256
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    if nbytes < ev_off + T * n * 8:
        raise RuntimeError("eks_yev_bytes smaller than the (T, n) y / ev planes")
    _lib.check(lib.eks_ensemble(d.data_ptr(), _lib.EKS_F64, 1, T, E, n, 0, n, T * n, 1, m,
                                buf.data_ptr(), buf.data_ptr() + ev_off, _lib.stream_ptr()),
               "eks_ensemble")
    planes = buf[:ev_off + T * n * 8]
    preds = planes[:T * n * 8].view(torch.float64).reshape(T, n).cpu().numpy()
    var = planes[ev_off:].view(torch.float64).reshape(T, n).cpu().numpy()
    return Yev(buf, 1, T, E, n, code, mode), preds, var


def ensemble(markers_list, keys, mode: str = "median"):
    """eks/ensemble_kalman.py:4-57, same 6-tuple:
    (ensemble_preds (T,n), ensemble_vars (T,n), ensemble_stacks (E,T,n),
     keypoints_avg_dict, keypoints_var_dict, keypoints_stack_dict)."""
    if mode not in ("median", "mean"):
        raise ValueError(f"{mode} averaging not supported")
    n_models = len(markers_list)
    T = markers_list[0].shape[0]
    stack = np.zeros((n_models, T, len(keys)))
    for e, df in enumerate(markers_list):
        for j, key in enumerate(keys):
            stack[e, :, j] = df[key]
    preds, var = ensemble_array(stack, mode)
    avg_d = {k: preds[:, j] for j, k in enumerate(keys)}
    var_d = {k: var[:, j] for j, k in enumerate(keys)}
    stack_d = defaultdict(dict)
    for e in range(n_models):
        for j, k in enumerate(keys):
            stack_d[e][k] = stack[e, :, j]
    return preds, var, stack, avg_d, var_d, stack_d


# --------------------------------------------------------------------------
def _forward(y, m0, S0, C, R, A, Q, ensemble_vars, want_outputs=True):
    torch = _lib.require_gpu()
    y = np.asarray(y, dtype=np.float64)
    ev = np.asarray(ensemble_vars, dtype=np.float64)
    T, n = y.shape
    r = np.asarray(m0).shape[0]
    # the reference writes R[i, i] = ev[t, i] only for i < ev.shape[1]
    # (:88-89); the rest of R, off-diagonals included, is used as given.
    ev_full = np.empty((T, n))
    R_np = np.asarray(R, dtype=np.float64)
    ev_full[:] = np.diag(R_np)[None, :]
    ev_full[:, :ev.shape[1]] = ev[:T]
    Roff = R_np.copy()
    np.fill_diagonal(Roff, 0.0)
    has_off = bool(np.any(Roff != 0))
    dev = {k: _to_dev(v, torch) for k, v in
           dict(y=y, ev=ev_full, m0=m0, S0=S0, A=A, Q=Q, C=C).items()}
    Rd = _to_dev(Roff, torch) if has_off else None
    mf = torch.empty((T, r), dtype=torch.float64, device="cuda")
    Vf = torch.empty((T, r, r), dtype=torch.float64, device="cuda")
    S = torch.empty((T, r, r), dtype=torch.float64, device="cuda")
    nll = torch.empty((1,), dtype=torch.float64, device="cuda")
    status = torch.empty((1,), dtype=torch.int32, device="cuda")
    lib = _lib.load()
    _lib.check(lib.eks_forward(1, T, n, r, dev["y"].data_ptr(), dev["ev"].data_ptr(),
                               dev["m0"].data_ptr(), dev["S0"].data_ptr(), dev["A"].data_ptr(),
                               dev["Q"].data_ptr(), dev["C"].data_ptr(),
                               Rd.data_ptr() if Rd is not None else None, 1,
                               mf.data_ptr(), Vf.data_ptr(), S.data_ptr(), nll.data_ptr(),
                               status.data_ptr(), _lib.stream_ptr()), "eks_forward")
    _raise_if_singular(status.cpu().numpy(), "filtering_pass")
    return mf.cpu().numpy(), Vf.cpu().numpy(), S.cpu().numpy(), float(nll.cpu()[0])


def filtering_pass(y, m0, S0, C, R, A, Q, ensemble_vars):
    """eks/ensemble_kalman.py:59-107 -> (mf (T,r), Vf (T,r,r), S (T,r,r)).

    As in the reference, ``R``'s diagonal is overwritten in place (it ends
    holding ensemble_vars[T-1]) and S[T-1] is left at zero."""
    mf, Vf, S, _ = _forward(y, m0, S0, C, R, A, Q, ensemble_vars)
    ev = np.asarray(ensemble_vars)
    T = np.asarray(y).shape[0]
    for i in range(ev.shape[1]):  # in-place side effect of :88-89 / :99-100
        R[i, i] = ev[T - 1][i]
    return mf, Vf, S


forward_pass = filtering_pass


def compute_nll(y, m0, S0, C, A, Q, ensemble_vars, R=None):
    """Gaussian innovation NLL of the forward filter:
    1/2 sum_t [n log 2pi + log det Sigma_t + e_t^T Sigma_t^-1 e_t] with
    Sigma_t = R_t + C P_t C^T, e_t = y_t - C m_t (P_t, m_t the predicted
    covariance / mean; t = 0 uses m0, S0).  R defaults to the identity
    placeholder the wrappers pass, whose diagonal is replaced by the
    ensemble variances."""
    n = np.asarray(y).shape[1]
    R = np.eye(n) if R is None else np.array(R, dtype=np.float64)
    return _forward(y, m0, S0, C, R, A, Q, ensemble_vars)[3]


def kalman_dot(array, V, C, R):
    """eks/ensemble_kalman.py:110-117: V C^T (R + C V C^T)^-1 array."""
    torch = _lib.require_gpu()
    x = np.asarray(array, dtype=np.float64)
    vec = x.ndim == 1
    x2 = x[:, None] if vec else x
    n, k = x2.shape
    r = np.asarray(V).shape[0]
    d = {kk: _to_dev(v, torch) for kk, v in dict(x=x2, V=V, C=C, R=R).items()}
    out = torch.empty((r, k), dtype=torch.float64, device="cuda")
    status = torch.empty((1,), dtype=torch.int32, device="cuda")
    lib = _lib.load()
    _lib.check(lib.eks_kalman_dot(n, r, k, d["x"].data_ptr(), d["V"].data_ptr(),
                                  d["C"].data_ptr(), d["R"].data_ptr(), out.data_ptr(),
                                  status.data_ptr(), _lib.stream_ptr()), "eks_kalman_dot")
    _raise_if_singular(status.cpu().numpy(), "kalman_dot")
    o = out.cpu().numpy()
    return o[:, 0] if vec else o


def smooth_backward(y, mf, Vf, S, A, Q=None, C=None):
    """eks/ensemble_kalman.py:120-164 -> (ms (T,r), Vs (T,r,r), CV (T-1,r,r)).
    ``Q`` and ``C`` are unused and ``y`` only supplies T, as in the reference."""
    torch = _lib.require_gpu()
    T = np.asarray(y).shape[0] if y is not None else np.asarray(mf).shape[0]
    mf = np.asarray(mf, dtype=np.float64)[:T]
    r = mf.shape[1]
    d = {k: _to_dev(v, torch) for k, v in
         dict(mf=mf, Vf=np.asarray(Vf)[:T], S=np.asarray(S)[:T], A=A).items()}
    ms = torch.empty((T, r), dtype=torch.float64, device="cuda")
    Vs = torch.empty((T, r, r), dtype=torch.float64, device="cuda")
    CV = torch.empty((max(T - 1, 1), r, r), dtype=torch.float64, device="cuda")
    status = torch.empty((1,), dtype=torch.int32, device="cuda")
    lib = _lib.load()
    _lib.check(lib.eks_backward(1, T, r, d["mf"].data_ptr(), d["Vf"].data_ptr(),
                                d["S"].data_ptr(), d["A"].data_ptr(), 1, ms.data_ptr(),
                                Vs.data_ptr(), CV.data_ptr(), status.data_ptr(),
                                _lib.stream_ptr()), "eks_backward")
    _raise_if_singular(status.cpu().numpy(), "smooth_backward")
    return ms.cpu().numpy(), Vs.cpu().numpy(), CV.cpu().numpy()[:max(T - 1, 0)]


backward_pass = smooth_backward
