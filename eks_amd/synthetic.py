"""Seeded synthetic ensemble-prediction generators.

All values are rounded to float32 so that float32 device storage is lossless;
host-side checkers read the same values as float64.

Shapes use the reference's vocabulary: E ensemble members, T frames,
K keypoints, V cameras, D = 2 coordinates (x, y).
"""
from __future__ import annotations

import numpy as np


def singleview_obs(rng: np.random.Generator, E: int, T: int, K: int = 1,
                   walk_sigma: float = 2.0, outlier_frac: float = 0.01,
                   outlier_px: float = 30.0) -> np.ndarray:
    """(E, T, K, 2) float32 member predictions of K 2-D keypoints.

    Latent: Gaussian random walk (sigma ``walk_sigma`` px per frame) starting
    at U(50, 450).  Member e observes it with N(0, sigma_e^2) noise,
    sigma_e ~ U(0.5, 3) px (per member and keypoint); a fraction
    ``outlier_frac`` of (t, e) pairs is displaced by ``outlier_px``.
    """
    start = rng.uniform(50.0, 450.0, size=(1, K, 2))
    steps = rng.normal(0.0, walk_sigma, size=(T, K, 2))
    steps[0] = 0.0
    latent = start + np.cumsum(steps, axis=0)  # (T, K, 2)
    sig = rng.uniform(0.5, 3.0, size=(E, 1, K, 1))
    obs = latent[None] + rng.normal(0.0, 1.0, size=(E, T, K, 2)) * sig
    mask = rng.random(size=(E, T, K, 1)) < outlier_frac
    ang = rng.uniform(0.0, 2 * np.pi, size=(E, T, K, 1))
    disp = np.concatenate([np.cos(ang), np.sin(ang)], axis=-1) * outlier_px
    obs = obs + mask * disp
    return obs.astype(np.float32)


def multiview_obs(rng: np.random.Generator, V: int, E: int, T: int, K: int = 1,
                  walk_sigma: float = 0.02, outlier_frac: float = 0.01,
                  outlier_px: float = 30.0) -> np.ndarray:
    """(E, T, K, 2V) float32: a 3-D latent random walk seen by V cameras,
    each through a random 2x3 affine map with scale 50-150 px per unit."""
    latent = np.cumsum(rng.normal(0.0, walk_sigma, size=(T, K, 3)), axis=0)
    latent += rng.uniform(-1.0, 1.0, size=(1, K, 3))
    cols = []
    for _ in range(V):
        M = rng.normal(size=(K, 2, 3))
        M *= rng.uniform(50.0, 150.0, size=(K, 1, 1)) / np.linalg.norm(M, axis=2, keepdims=True)
        off = rng.uniform(150.0, 350.0, size=(1, K, 2))
        cols.append(np.einsum('kij,tkj->tki', M, latent) + off)
    clean = np.concatenate(cols, axis=-1)  # (T, K, 2V)
    sig = rng.uniform(0.5, 3.0, size=(E, 1, K, 2 * V))
    obs = clean[None] + rng.normal(size=(E, T, K, 2 * V)) * sig
    mask = rng.random(size=(E, T, K, 2 * V)) < outlier_frac
    obs = obs + mask * rng.choice([-outlier_px, outlier_px], size=obs.shape)
    return obs.astype(np.float32)


# Key order of the reference's pupil smoother (eks/pupil_smoother.py:102-103)
PUPIL_KEYS = ('pupil_top_r_x', 'pupil_top_r_y', 'pupil_bottom_r_x', 'pupil_bottom_r_y',
              'pupil_right_r_x', 'pupil_right_r_y', 'pupil_left_r_x', 'pupil_left_r_y')


def pupil_obs(rng: np.random.Generator, E: int, T: int, a: float = 0.99,
              centre=(16.0, 52.0, 51.0), noise_px: float = 1.0) -> np.ndarray:
    """(E, T, 8) float32 pupil keypoints (PUPIL_KEYS order).

    Latent (diameter, com_x, com_y) is AR(1) with coefficient ``a`` around
    ``centre`` (magnitudes from data/misc/pupil-test); keypoints follow the
    measurement matrix of eks/pupil_smoother.py:150-153.
    """
    mu = np.asarray(centre)
    sd = np.array([1.5, 2.0, 2.0]) * np.sqrt(1 - a * a)
    from scipy.signal import lfilter
    noise = rng.normal(size=(T, 3)) * sd
    noise[0] = 0.0
    z = mu + lfilter([1.0], [1.0, -a], noise, axis=0)  # x_t = a x_{t-1} + w_t
    d, cx, cy = z[:, 0], z[:, 1], z[:, 2]
    clean = np.stack([cx, cy - d / 2, cx, cy + d / 2, cx + d / 2, cy, cx - d / 2, cy], axis=1)
    sig = rng.uniform(0.5, 1.5, size=(E, 1, 8)) * noise_px
    return (clean[None] + rng.normal(size=(E, T, 8)) * sig).astype(np.float32)
