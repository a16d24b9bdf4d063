"""Newton ("opti") forward filter -- module-path mirror of eks/newton_eks.py.

    kalman_newton_recursive(y, mu0, S0, A, B, ensemble_vars, E, max_iter=1)
        eks/newton_eks.py:115-148, numpy in / numpy out, computed by the
        k_newton HIP kernel (eks_newton_filter in include/eks_hip.h).
    newton_filter_batch(y, ev, mu0, S0, A, Bm, E, max_iter=1)
        the same for B trajectories held on the GPU (one lane each).

Semantics kept from the reference: q[0] = mu0 without a measurement update,
P starts as inv(S0), P carries over between iterations, the update is in
place so the returned loss vector (max_iter > 1) is all zeros, and a zero
ensemble variance or a singular S0 raises numpy.linalg.LinAlgError.
``hessian``/``gradient``/``schur_diag`` of the reference are unused research
prototypes (``gradient`` reads an undefined ``r``) and are not provided.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def _f64(torch, a):
    return torch.as_tensor(np.asarray(a, dtype=np.float64) if not torch.is_tensor(a) else a,
                           dtype=torch.float64, device="cuda").contiguous()


def newton_filter_batch(y, ev, mu0, S0, A, Bm, E, max_iter: int = 1):
    """y, ev: (B, T, n); model arrays either per trajectory ((B, r), (B, r, r),
    (B, n, r)) or shared ((r,), (r, r), (n, r)).  Returns (q (B, T, r) f64 on
    the GPU, status (B) int32) -- status bit EKS_STATUS_SINGULAR where the
    reference would raise."""
    torch = _lib.require_gpu()
    y = _f64(torch, y)
    ev = _f64(torch, ev)
    if y.dim() != 3 or ev.shape != y.shape:
        raise ValueError("y and ensemble_vars must both be (B, T, n)")
    Bn, T, n = y.shape
    mu0, S0, A, Bm, E = (_f64(torch, a) for a in (mu0, S0, A, Bm, E))
    shared = 1 if mu0.dim() == 1 else 0
    r = mu0.shape[-1]
    lead = () if shared else (Bn,)
    for name, a, shp in (("S0", S0, (r, r)), ("A", A, (r, r)), ("B", Bm, (n, r)),
                         ("E", E, (r, r))):
        if tuple(a.shape) != lead + shp:
            raise ValueError(f"{name} has shape {tuple(a.shape)}, expected {lead + shp}")
    q = torch.empty((Bn, T, r), dtype=torch.float64, device="cuda")
    status = torch.zeros(Bn, dtype=torch.int32, device="cuda")
    lib = _lib.load()
    _lib.check(lib.eks_newton_filter(Bn, T, n, r, y.data_ptr(), ev.data_ptr(), mu0.data_ptr(),
                                     S0.data_ptr(), A.data_ptr(), Bm.data_ptr(), E.data_ptr(),
                                     shared, int(max_iter), q.data_ptr(), status.data_ptr(),
                                     _lib.stream_ptr()), "eks_newton_filter")
    return q, status


def kalman_newton_recursive(y, mu0, S0, A, B, ensemble_vars, E, max_iter=1):
    """eks/newton_eks.py:115-148.  Returns q (T, r), or (q, loss) with
    loss = zeros(max_iter) when max_iter > 1 (the reference's return)."""
    y = np.asarray(y, dtype=np.float64)
    q, status = newton_filter_batch(y[None], np.asarray(ensemble_vars, dtype=np.float64)[None],
                                    mu0, S0, A, B, E, max_iter)
    if int(status[0].item()) != 0:
        raise np.linalg.LinAlgError("Singular matrix (kalman_newton_recursive)")
    q = q[0].cpu().numpy()
    if max_iter == 1:
        return q
    return q, np.zeros(max_iter)
