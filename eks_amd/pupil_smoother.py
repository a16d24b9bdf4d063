"""Module-path alias of the reference's eks/pupil_smoother.py."""
from .core import ensemble, filtering_pass, kalman_dot, smooth_backward  # noqa: F401
from .fit import pupil_centre as get_pupil_location  # noqa: F401
from .fit import pupil_diameter as get_pupil_diameter  # noqa: F401
from .newton_eks import kalman_newton_recursive  # noqa: F401
from .smoothers import (ensemble_kalman_smoother_pupil, eks_opti_smoother_pupil,  # noqa: F401
                        pupil_smoothing_sweep)
