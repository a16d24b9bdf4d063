"""Module-path alias of the reference's eks/multiview_pca_smoother.py."""
from .core import ensemble, filtering_pass, kalman_dot, smooth_backward  # noqa: F401
from .newton_eks import kalman_newton_recursive  # noqa: F401
from .smoothers import (ensemble_kalman_smoother_multi_cam, eks_opti_smoother_multi_cam,  # noqa: F401
                        ensemble_kalman_smoother_paw_asynchronous,
                        eks_opti_smoother_paw_asynchronous)
