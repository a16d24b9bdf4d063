"""Module-path alias of the reference's eks/ensemble_kalman.py."""
from .core import ensemble, filtering_pass, kalman_dot, smooth_backward  # noqa: F401
