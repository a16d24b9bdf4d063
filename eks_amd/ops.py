"""``torch.ops.eks.*``: the C ABI entry points as PyTorch operators registered
in C++ ("the torch extension wraps the same functions").

    import eks_amd.ops                       # loads libeks_torch.so
    preds, vars_ = torch.ops.eks.ensemble(obs, "median")
    mf, Vf, S, nll, status = torch.ops.eks.forward(y, ev, m0, S0, A, Q, C)
    ms, Vs, CV, status = torch.ops.eks.backward(mf, Vf, S, A)
    out, status = torch.ops.eks.smooth(obs, params, 2, 2, "median", 0, 0)

The operators are defined by ``TORCH_LIBRARY(eks, ...)`` in
``eks_amd/csrc/torch_ops.cpp`` (built into ``eks_amd/lib/libeks_torch.so`` by
``eks_amd.build``), each with a CUDA-key kernel that calls libeks_hip.so on
the current stream and a Meta kernel for shape propagation (FakeTensor /
``torch.compile``): no Python frame in their dispatch and no CPU kernel (a
CPU tensor is a dispatch error).  Layout conventions are those of
``eks_amd.batch``: obs is (B, T, E, n) with any strides.

    ensemble   eks/ensemble_kalman.py:4-57        forward   :59-117 (filtering_pass)
    backward   :120-164 (smooth_backward)          nll       compute_nll
    smooth     the fused hot path                  fit       eks/multiview_pca_smoother.py:684-731
    newton_filter  eks/newton_eks.py:115-148       interp1d  eks/multiview_pca_smoother.py:86-96
"""
from __future__ import annotations

import os

import torch

from . import _lib

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libeks_torch.so")

OPS = ("ensemble", "forward", "backward", "smooth", "nll", "fit", "newton_filter", "interp1d")


def _load():
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} is missing: build it (python -m eks_amd.build). "
                           "eks_amd has no CPU fallback.")
    _lib.load()  # libeks_hip.so first (libeks_torch.so links it)
    torch.ops.load_library(LIB)


_load()
