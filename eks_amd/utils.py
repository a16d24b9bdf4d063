"""DLC / Lightning-Pose DataFrame helpers (eks/utils.py:1-22 of the reference)."""
from __future__ import annotations

import pandas as pd

TRACKER = "ensemble-kalman_tracker"


def make_dlc_pandas_index(keypoint_names):
    """(scorer='ensemble-kalman_tracker', bodyparts, coords in x/y/likelihood)
    column index of the output DataFrames (eks/utils.py:4-10)."""
    return pd.MultiIndex.from_product([[TRACKER], list(keypoint_names), ["x", "y", "likelihood"]],
                                      names=["scorer", "bodyparts", "coords"])


def convert_lp_dlc(df_lp, keypoint_names, model_name=None):
    """Flatten a 3-level LP/DLC frame to '{kp}_{x|y|likelihood}' columns
    (eks/utils.py:13-22)."""
    cols = {}
    for kp in keypoint_names:
        for c in ("x", "y", "likelihood"):
            key = (kp, c) if model_name is None else (model_name, kp, c)
            cols[f"{kp}_{c}"] = df_lp.loc[:, key]
    return pd.DataFrame(cols, index=df_lp.index)
