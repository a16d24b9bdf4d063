"""eks_amd -- MI355X-native ensemble Kalman smoother.

Drop-in for the hot path of erialc-cal/eks (ensemble -> filtering_pass ->
smooth_backward -> projection): the recursions run as hand-written HIP
kernels for gfx950 (libeks_hip.so, C ABI in include/eks_hip.h), bound here
with ctypes.  There is no CPU fallback.

    eks_amd.core       ensemble, filtering_pass, kalman_dot, smooth_backward,
                       forward_pass, backward_pass, compute_nll (numpy API)
    eks_amd.batch      device-resident batched fused smoother (torch tensors)
    eks_amd.smoothers  multi-camera / pupil / single-view entry points
    eks_amd.fit        per-keypoint model fitting done before the smoother
"""
from . import core, utils  # noqa: F401
from .core import (backward_pass, compute_nll, ensemble, filtering_pass,  # noqa: F401
                   forward_pass, kalman_dot, smooth_backward)

__version__ = "0.1.0"
