"""Model fitting that precedes the smoother (host side, per keypoint).

These are the steps the reference's wrappers run between ``ensemble`` and
``filtering_pass``.  They reduce over
the time axis once per trajectory and are small next to the recursions;
the recursions themselves run in the HIP kernels.

    singleview_model   build definition
    multicam_model     eks/multiview_pca_smoother.py:684-731
    pupil_model        eks/pupil_smoother.py:101-172
"""
from __future__ import annotations

import warnings

import numpy as np

PUPIL_KEYS = ('pupil_top_r_x', 'pupil_top_r_y', 'pupil_bottom_r_x', 'pupil_bottom_r_y',
              'pupil_right_r_x', 'pupil_right_r_y', 'pupil_left_r_x', 'pupil_left_r_y')
# measurement matrix of eks/pupil_smoother.py:150-153 (rows in PUPIL_KEYS order)
PUPIL_C = np.array([[0, 1, 0], [-.5, 0, 1], [0, 1, 0], [.5, 0, 1],
                    [.5, 1, 0], [0, 0, 1], [-.5, 1, 0], [0, 0, 1]], dtype=np.float64)


def low_variance_frames(ens_vars: np.ndarray, quantile_keep: float) -> np.ndarray:
    """Indices of frames whose largest ensemble variance is at or below the
    ``quantile_keep`` percentile (linear interpolation), as
    eks/multiview_pca_smoother.py:685-688."""
    worst = ens_vars.max(axis=1)
    return np.flatnonzero(worst <= np.percentile(worst, quantile_keep))


def _step_cov(z_good: np.ndarray, smooth_param: float) -> np.ndarray:
    """Q = s * cov(successive differences of the kept frames), ddof = 1
    (eks/multiview_pca_smoother.py:726-728)."""
    d = np.diff(z_good, axis=0)
    return smooth_param * np.atleast_2d(np.cov(d.T))


def singleview_model(preds, ens_vars, smooth_param, quantile_keep):
    """Single-view parameterisation: the multicam template
    without PCA -- C = A = I2, m0 = 0, S0 = diag(var of kept frames),
    Q = s cov(diff(kept frames)), offset = mean of kept frames."""
    keep = low_variance_frames(ens_vars, quantile_keep)
    offset = preds[keep].mean(axis=0)
    z = preds[keep] - offset
    return dict(m0=np.zeros(2), S0=np.diag(z.var(axis=0)), A=np.eye(2),
                Q=_step_cov(z, smooth_param), C=np.eye(2), offset=offset, keep=keep)


def principal_axes(X: np.ndarray, k: int):
    """Top-k principal axes of the rows of X (eigen-decomposition of the
    sample covariance, as sklearn's PCA 'covariance_eigh' solver).  Row i of
    the result is axis i; signs are arbitrary (outputs do not depend on them
    because S0 is diagonal)."""
    Xc = X - X.mean(axis=0)
    w, v = np.linalg.eigh(Xc.T @ Xc / max(len(X) - 1, 1))
    top = np.argsort(w)[::-1][:k]
    return v[:, top].T, X.mean(axis=0)


def multicam_model(preds, ens_vars, smooth_param, quantile_keep, n_latent=3):
    """eks/multiview_pca_smoother.py:684-731 for one keypoint seen by V
    cameras: preds / ens_vars are (T, 2V) (camera-major x, y columns)."""
    keep = low_variance_frames(ens_vars, quantile_keep)
    offset = preds[keep].mean(axis=0)
    y = preds - offset
    axes, centre = principal_axes(y[keep], n_latent)
    z_keep = (y[keep] - centre) @ axes.T
    r = n_latent
    return dict(m0=np.zeros(r), S0=np.diag(z_keep.var(axis=0)), A=np.eye(r),
                Q=_step_cov(z_keep, smooth_param), C=axes.T.copy(), offset=offset, keep=keep)


def pupil_centre(cols) -> np.ndarray:
    """Pupil centre of mass from the four keypoints (eks/pupil_smoother.py:14-39)."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", category=RuntimeWarning)
        top = np.stack([cols['pupil_top_r_x'], cols['pupil_top_r_y']], 1)
        bot = np.stack([cols['pupil_bottom_r_x'], cols['pupil_bottom_r_y']], 1)
        lef = np.stack([cols['pupil_left_r_x'], cols['pupil_left_r_y']], 1)
        rig = np.stack([cols['pupil_right_r_x'], cols['pupil_right_r_y']], 1)
        x_tb = np.nanmedian(np.stack([top[:, 0], bot[:, 0]], 1), axis=1)   # either may be NaN
        x_lr = np.median(np.stack([rig[:, 0], lef[:, 0]], 1), axis=1)      # both needed
        y_tb = np.median(np.stack([top[:, 1], bot[:, 1]], 1), axis=1)      # both needed
        y_lr = np.nanmedian(np.stack([rig[:, 1], lef[:, 1]], 1), axis=1)   # either may be NaN
        return np.stack([np.nanmedian(np.stack([x_tb, x_lr], 1), axis=1),
                         np.nanmedian(np.stack([y_tb, y_lr], 1), axis=1)], 1)


def pupil_diameter(cols) -> np.ndarray:
    """Median of six diameter estimates: top-bottom, left-right and four
    neighbour pairs scaled by sqrt 2 (eks/pupil_smoother.py:42-68)."""
    p = {k: np.stack([cols[f'pupil_{k}_r_x'], cols[f'pupil_{k}_r_y']])
         for k in ('top', 'bottom', 'left', 'right')}
    ests = [np.linalg.norm(p['top'] - p['bottom'], axis=0),
            np.linalg.norm(p['left'] - p['right'], axis=0)]
    ests += [np.linalg.norm(p[a] - p[b], axis=0) * 2 ** 0.5
             for a, b in (('top', 'left'), ('top', 'right'), ('bottom', 'left'), ('bottom', 'right'))]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", category=RuntimeWarning)
        return np.nanmedian(ests, axis=0)


def pupil_model(preds, state_transition_matrix):
    """eks/pupil_smoother.py:109-172: latent (diameter, com_x, com_y)."""
    A = np.asarray(state_transition_matrix, dtype=np.float64)
    cols = {k: preds[:, j] for j, k in enumerate(PUPIL_KEYS)}
    com = pupil_centre(cols)
    diam = pupil_diameter(cols)
    mx, my = com[:, 0].mean(), com[:, 1].mean()
    var = np.array([diam.var(), (com[:, 0] - mx).var(), (com[:, 1] - my).var()])
    return dict(m0=np.array([diam.mean(), 0.0, 0.0]), S0=np.diag(var), A=A,
                Q=np.diag(var * (1 - np.diag(A) ** 2)), C=PUPIL_C.copy(),
                offset=np.array([mx, my] * 4), mx=mx, my=my)


def paw_async_models(cam_preds, cam_vars, smooth_param, quantile_keep):
    """Model fit of the asynchronous paw smoother
    (eks/multiview_pca_smoother.py:124-241).  cam_preds / cam_vars: (2, T, 4)
    ensemble outputs of the left and the right (resampled, flipped) camera,
    columns (paw 1 x, y, paw 2 x, y).  One PCA subspace is fitted on the good
    frames of both paws stacked (2 rows per frame); each paw gets its own S0
    and Q from its principal components.  Returns ([model paw 1, model paw
    2], None); each model carries its centred observations 'y' and variances
    'ev' (left view x, y, right view x, y)."""
    lp, rp = cam_preds
    lv, rv = cam_vars
    worst = np.max(np.hstack([lv, rv]), 1)
    good = np.flatnonzero(worst <= np.percentile(worst, quantile_keep))
    stacked = np.empty((2 * len(good), 4))
    stacked[0::2] = np.hstack([lp[good][:, :2], rp[good][:, :2]])
    stacked[1::2] = np.hstack([lp[good][:, 2:4], rp[good][:, 2:4]])
    means = stacked.mean(axis=0)
    axes, centre = principal_axes(stacked - means, 3)
    models = []
    for k in range(2):
        pred = np.hstack([lp[:, 2 * k:2 * k + 2], rp[:, 2 * k:2 * k + 2]])
        var = np.hstack([lv[:, 2 * k:2 * k + 2], rv[:, 2 * k:2 * k + 2]])
        y = pred - means
        z_good = ((y - centre) @ axes.T)[good]
        models.append(dict(m0=np.zeros(3), S0=np.diag(z_good.var(axis=0)), A=np.eye(3),
                           Q=_step_cov(z_good, smooth_param), C=axes.T.copy(), offset=means,
                           y=y, ev=var))
    return models, None
