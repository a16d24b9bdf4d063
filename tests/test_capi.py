"""CPU-side checks of the C ABI: the library loads, exports exactly what
include/eks_hip.h declares, and rejects bad arguments before touching the
GPU.  No kernel is launched here (there is no GPU in the build container)."""
import ctypes

import pytest

from eks_amd import _lib


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    declared = _lib.header_symbols()
    assert len(declared) >= 10
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/eks_hip.h but not exported"
    # and the ctypes signature table covers every declared symbol
    assert set(declared) == set(_lib.SIGNATURES)


def test_limits_and_sizes():
    lib = _lib.load()
    assert lib.eks_version() >= 100
    assert lib.eks_max_latent() >= 3 and lib.eks_max_obs() >= 8 and lib.eks_max_members() >= 8
    for n, r in [(2, 2), (8, 3), (4, 3)]:
        assert lib.eks_param_len(n, r) == r + 3 * r * r + n * r + n
    assert lib.eks_smooth_workspace_bytes(10, 100, 2, 2, 5, 1) >= 10 * 100 * 5 * 8
    # time-parallel plan: few long trajectories are cut into chunks
    L = lib.eks_smooth_chunk_len(17, 100000, 2)
    assert 16 <= L < 100000 and L % 8 == 0
    assert lib.eks_smooth_chunk_len(1 << 20, 1000, 2) == 0  # enough trajectories: sequential
    # automatic algorithm: two-pass for many single-view trajectories, the
    # three-pass scan for few or multi-view ones, sequential for very many
    assert lib.eks_smooth_algo(17408, 10000, 2, 2, 5, 0) == 3
    assert lib.eks_smooth_algo(17, 100000, 2, 2, 5, 0) == 2
    assert lib.eks_smooth_algo(17408, 10000, 8, 3, 5, 0) == 2
    assert lib.eks_smooth_algo(1 << 20, 1000, 2, 2, 5, 0) == 1
    assert lib.eks_smooth_algo(17408, 10000, 2, 2, 11, 3) == 2  # E = 11: no algo-3 kernels
    assert lib.eks_smooth_algo(4, 100, 2, 2, 5, 9) == 0
    # shapes without compiled kernels (five cameras: n = 10) run the runtime-n kernel
    assert lib.eks_smooth_algo(17, 50000, 10, 3, 5, 0) == 4
    assert lib.eks_smooth_algo(17, 50000, 8, 3, 5, 4) == 4
    # ... sequential for many trajectories, time-parallel (chunk planes) for few
    assert lib.eks_smooth_workspace_bytes(1 << 20, 100, 10, 3, 5, 0) == (1 << 20) * 100 * 9 * 8
    assert lib.eks_smooth_workspace_bytes(17, 1000, 10, 3, 5, 0) > 17 * 1000 * 10 * 16
    assert lib.eks_smooth_workspace_bytes(17, 100000, 2, 2, 5, 2) >= 17 * 100000 * 2 * 16


def test_argument_errors_do_not_launch():
    lib = _lib.load()
    rc = lib.eks_smooth(None, 0, 1, 10, 5, 2, 2, 0, 0, 0, 0, 0, None, None, 0, 0, 0,
                        None, None, None, 0, 0, 0, None, None)
    assert rc == _lib.EKS_ERR_ARG
    assert b"NULL" in lib.eks_last_error()
    rc = lib.eks_ensemble(ctypes.c_void_p(8), 0, 1, 10, 5, 2, 0, 0, 0, 0, 7,
                          ctypes.c_void_p(8), ctypes.c_void_p(8), None)
    assert rc == _lib.EKS_ERR_ARG and b"averaging not supported" in lib.eks_last_error()
    with pytest.raises(_lib.EksError):
        _lib.check(rc, "eks_ensemble")


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import numpy as np
    from eks_amd import core
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        core.filtering_pass(np.zeros((3, 2)), np.zeros(2), np.eye(2), np.eye(2), np.eye(2),
                            np.eye(2), np.eye(2), np.ones((3, 2)))


def test_product_package_never_imports_oracle():
    import glob
    import os
    root = os.path.dirname(_lib.HERE)
    for path in glob.glob(os.path.join(root, "eks_amd", "**", "*.py"), recursive=True):
        src = open(path).read()
        assert "oracle" not in src.replace("oracle/", ""), f"{path} references the oracle"


def test_torch_ops_registered_with_fake_shapes():
    """torch.ops.eks.* exist and propagate shapes without a GPU;
    calling them on CPU tensors fails loudly (no CPU fallback)."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    import eks_amd.ops as ops
    for name in ops.OPS:
        assert hasattr(torch.ops.eks, name)
    with FakeTensorMode():
        obs = torch.empty((3, 100, 5, 2), dtype=torch.float32)
        params = torch.empty((3, 20), dtype=torch.float64)  # eks_param_len(2, 2)
        out, st = torch.ops.eks.smooth(obs, params, 2, 2, "median", 0, 0)
        assert out.shape == (3, 100, 2) and out.dtype == torch.float64 and st.shape == (3,)
        p, s = torch.ops.eks.ensemble(obs, "median")
        assert p.shape == (3, 100, 2)
        prm, _ = torch.ops.eks.fit(obs, "singleview", 2, 2, 0.01, 25.0, "median")
        assert prm.shape == (3, 20)
        assert torch.ops.eks.nll(obs, params, 2, 2, "median", 0).shape == (3,)
    # no CPU kernel is registered (csrc/torch_ops.cpp): a dispatch error
    with pytest.raises(NotImplementedError, match="CPU"):
        torch.ops.eks.ensemble(torch.zeros((1, 4, 3, 2)), "median")


def test_header_enums_match_bindings():
    """Every enum constant the header defines has the same value in _lib."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(_lib.__file__), "..", "include", "eks_hip.h")).read()
    consts = dict(re.findall(r"\b(EKS_[A-Z0-9_]+)\s*=\s*(-?\d+)", hdr))
    assert "EKS_MODEL_PUPIL" in consts
    for name, val in consts.items():
        if hasattr(_lib, name):
            assert getattr(_lib, name) == int(val), name


def test_model_flags_pupil_structure():
    """batch.model_flags: the pupil promise needs C = the pupil matrix
    (eks/pupil_smoother.py:150-153) and diagonal A and Q."""
    import numpy as np
    from eks_amd import batch, fit
    A = np.diag([0.99, 0.999, 0.999])
    Q = np.diag([1.0, 2.0, 3.0])
    assert batch.model_flags(A, fit.PUPIL_C, Q) == _lib.EKS_MODEL_PUPIL
    assert batch.model_flags(np.stack([A, A]), np.stack([fit.PUPIL_C] * 2),
                             np.stack([Q, Q])) == _lib.EKS_MODEL_PUPIL
    assert batch.model_flags(A, fit.PUPIL_C) == 0           # Q unknown: no promise
    Qb = Q.copy()
    Qb[0, 1] = 1e-3
    assert batch.model_flags(A, fit.PUPIL_C, Qb) == 0
    Cb = fit.PUPIL_C.copy()
    Cb[1, 0] = -0.49
    assert batch.model_flags(A, Cb, Q) == 0
    assert batch.model_flags(np.eye(3), fit.PUPIL_C, Q) == (_lib.EKS_MODEL_A_IDENTITY
                                                           | _lib.EKS_MODEL_PUPIL)
    # the pupil model the wrappers fit
    preds = np.random.default_rng(0).normal(50, 2, size=(400, 8))
    m = fit.pupil_model(preds, np.diag([0.9, 0.99, 0.99]))
    assert batch.model_flags(m["A"], m["C"], m["Q"]) == _lib.EKS_MODEL_PUPIL


def test_fit_sizes_and_debug_keys():
    """eks_fit covers even n up to 16 (n > 8: the wide kernels); the debug
    keys round-trip their values (no GPU work: host globals only)."""
    lib = _lib.load()
    for n in (2, 4, 8, 10, 12, 16):
        assert lib.eks_fit_workspace_bytes(17, 5000, n) > 17 * 5000 * 8
    assert lib.eks_fit_workspace_bytes(17, 5000, 18) == 0
    # the wide fit's partial rows (2 + 4n + n(n + 1) doubles) are larger
    assert lib.eks_fit_workspace_bytes(17, 5000, 16) > lib.eks_fit_workspace_bytes(17, 5000, 8)
    for key, val in ((_lib.EKS_DBG_A3_LB, 2), (_lib.EKS_DBG_RT_FORM, 1), (_lib.EKS_DBG_FIT_SELECT, 2),
                     (_lib.EKS_DBG_A3_MODE, 1)):
        prev = _lib.debug_set(key, val)
        assert _lib.debug_set(key, prev) == val
    # the runtime-n workspace covers both forms once the time-parallel one is forced
    prev = _lib.debug_set(_lib.EKS_DBG_RT_FORM, 2)
    try:
        forced = lib.eks_smooth_workspace_bytes(1 << 20, 100, 10, 3, 5, 0)
    finally:
        _lib.debug_set(_lib.EKS_DBG_RT_FORM, prev)
    assert forced > lib.eks_smooth_workspace_bytes(1 << 20, 100, 10, 3, 5, 0)
