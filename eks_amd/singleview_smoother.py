"""Single-view smoother module (upstream eks name; absent from the snapshot)."""
from .smoothers import ensemble_kalman_smoother_single_view  # noqa: F401
