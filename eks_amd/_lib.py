"""ctypes binding of libeks_hip.so (the C ABI in include/eks_hip.h).

The HIP library is the product: there is no CPU fallback.  Loading fails with
an ImportError-style RuntimeError naming the missing file, and every compute
call requires a visible GPU (``torch.cuda.is_available()``).
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# EKS_LIB overrides the library path (kernel tuning experiments only)
LIB_PATH = os.environ.get("EKS_LIB") or os.path.join(HERE, "lib", "libeks_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "eks_hip.h")
HEADERS = [HEADER, os.path.join(os.path.dirname(HERE), "include", "eks_io.h")]

EKS_OK, EKS_ERR_ARG, EKS_ERR_UNSUPPORTED, EKS_ERR_HIP = 0, 1, 2, 4
EKS_STATUS_SINGULAR, EKS_STATUS_BAD_MODEL, EKS_STATUS_SCAN = 1, 2, 4
EKS_MODEL_A_IDENTITY, EKS_MODEL_C_IDENTITY, EKS_MODEL_PUPIL = 1, 2, 4
EKS_FIT_SINGLEVIEW, EKS_FIT_MULTICAM = 1, 2
EKS_F32, EKS_F64 = 0, 1
EKS_YEV32, EKS_YEV64 = 2, 3
EKS_MEDIAN, EKS_MEAN = 0, 1
EKS_DBG_WAIT_US, EKS_DBG_A3_SLICE_BYTES, EKS_DBG_FIT_SELECT, EKS_DBG_A3_MODE = 1, 2, 3, 4
EKS_DBG_A3_LB = 5
EKS_DBG_RT_FORM = 6

_p = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int
_sz = C.c_size_t

# argument types of every exported entry point (order as in the header)
SIGNATURES = {
    "eks_last_error": (C.c_char_p, []),
    "eks_version": (_i32, []),
    "eks_max_latent": (_i32, []),
    "eks_max_obs": (_i32, []),
    "eks_max_members": (_i32, []),
    "eks_ensemble": (_i32, [_p, _i32, _i64, _i64, _i32, _i32, _i64, _i64, _i64, _i64, _i32,
                            _p, _p, _p]),
    "eks_forward": (_i32, [_i64, _i64, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _i32,
                           _p, _p, _p, _p, _p, _p]),
    "eks_backward": (_i32, [_i64, _i64, _i32, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _p]),
    "eks_kalman_dot": (_i32, [_i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p]),
    "eks_param_len": (_i64, [_i32, _i32]),
    "eks_smooth_workspace_bytes": (_sz, [_i64, _i64, _i32, _i32, _i32, _i32]),
    "eks_smooth": (_i32, [_p, _i32, _i64, _i64, _i32, _i32, _i32, _i64, _i64, _i64, _i64, _i32,
                          _p, _p, _i64, _i64, _i64, _p, _p, _p, _sz, _i32, _i32, _p, _p]),
    "eks_smooth_chunk_len": (_i64, [_i64, _i64, _i32]),
    "eks_smooth_algo": (_i32, [_i64, _i64, _i32, _i32, _i32, _i32]),
    "eks_smooth_seg_workspace_bytes": (_sz, [_i64, _i64, _i32, _i32]),
    "eks_smooth_seg": (_i32, [_p, _i32, _i64, _i64, _i32, _i32, _i32, _i64, _i64, _i64, _i64,
                              _i32, _p, _p, _i64, _i64, _i64, _p, _p, _p, _sz, _i32, _p, _i64,
                              _i64, _i32, _p, _p, _p]),
    "eks_seg_combine": (_i32, [_i32, _i64, _i32, _i32, _i32, _p, _p, _p, _p]),
    "eks_newton_filter": (_i32, [_i64, _i64, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _i32, _i32,
                                 _p, _p, _p]),
    "eks_fit_workspace_bytes": (_sz, [_i64, _i64, _i32]),
    "eks_fit": (_i32, [_p, _i32, _i64, _i64, _i32, _i32, _i32, _i64, _i64, _i64, _i64, _i32, _i32,
                       C.c_double, C.c_double, _p, _p, _sz, _p, _p, _p]),
    "eks_yev_dtype": (_i32, [_i32, _i32, _i32]),
    "eks_yev_bytes": (_sz, [_i64, _i64, _i32, _i32, _i32, _i32]),
    "eks_interp1d": (_i32, [_p, _i64, _p, _i64, _i64, _i64, _p, _i64, _p, _i64, _i64, _p, _p]),
    "eks_debug_set": (_i64, [_i32, _i64]),
    "eks_profile_begin": (_i32, [_i32]),
    # include/eks_io.h (host-only)
    "eks_io_last_error": (C.c_char_p, []),
    "eks_csv_probe": (_i32, [C.c_char_p, _i32, _p, _p, _p]),
    "eks_csv_read": (_i32, [C.c_char_p, _i32, _p, _i64, _i64, _p, _p, _i64, _i32]),
    "eks_profile_end": (_i32, [_p, _p, _i32, _i32]),
}


def debug_set(key: int, value: int) -> int:
    """eks_debug_set (tests only): returns the previous value."""
    return int(load().eks_debug_set(key, value))


def profile_begin(max_calls: int) -> None:
    check(load().eks_profile_begin(max_calls), "eks_profile_begin")


def profile_end(max_kernels: int = 32):
    """[(kernel name, total ms)] over the profiled calls (eks_smooth, eks_fit)."""
    ms = (C.c_double * max_kernels)()
    names = C.create_string_buffer(64 * max_kernels)
    k = load().eks_profile_end(ms, names, max_kernels, 64)
    if k < 0:
        check(k, "eks_profile_end")
    raw = names.raw
    return [(raw[i * 64:(i + 1) * 64].split(b"\0")[0].decode(), ms[i]) for i in range(k)]

_lib = None


class EksError(RuntimeError):
    """A libeks_hip call returned an error code."""


def header_symbols() -> list[str]:
    """Function names declared in include/eks_hip.h and include/eks_io.h."""
    src = "\n".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(eks_[a-z_0-9]+)\s*\(", src)))


def load():
    """Load (once) and return the ctypes library handle."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            f"(python -m eks_amd.build, or __graft_entry__.build()). "
            f"eks_amd has no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("EKS_LIB") and not hasattr(lib, name):
            continue  # a tuning variant built from an older tree (tools/)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(code: int, what: str) -> None:
    if code != EKS_OK:
        msg = load().eks_last_error().decode(errors="replace")
        raise EksError(f"{what} failed (code {code}): {msg}")


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("eks_amd needs an AMD GPU (MI355X / gfx950): no HIP device is "
                           "visible, and there is no CPU fallback")
    return torch


def stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)
