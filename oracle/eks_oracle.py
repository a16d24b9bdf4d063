"""CPU oracle for the ensemble Kalman smoother hot path.

TEST INFRASTRUCTURE ONLY.  This module is the *checker*: it may be imported by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` and nowhere else.  The product package ``eks_amd`` never imports
it; its hot path runs the HIP kernels in ``eks_amd/csrc`` and fails loudly if
they are missing.

It is a plain-numpy restatement of the reference algorithm
(erialc-cal/eks snapshot at ``/root/reference``), written fresh.  Each function
cites the reference ``file:line`` whose behaviour it reproduces, including the
quirks SURVEY.md §8(a) lists (R mutated in place, ``S[T-1]`` left at zero,
variance divided by E even in median mode, Q and C unused by the backward
pass).  The per-timestep loops deliberately keep the reference's structure
(one dense ``np.linalg.solve`` per gain application) so that timing this module
is a fair stand-in for timing the reference.

Pinning: ``tests/test_oracle.py`` checks this module against
  * golden vectors produced by importing the reference itself in the build
    container (``tools/gen_golden.py`` -> ``tests/golden/*.npz``), and
  * the reference's own committed outputs (``data/mirror-mouse/output/eks.csv``,
    ``data/misc/pupil-test/kalman_smoothed_*.csv``, mirror-fish ``eks``
    outputs), sub-sampled into ``tests/golden/``.

``compute_nll`` and the single-view parameterisation have no counterpart in the
reference snapshot; they are this build's own
definitions.  The single-view fit is pinned by running the reference's
``ensemble``/``filtering_pass``/``smooth_backward`` on those definitions in
``tools/gen_golden.py``; the NLL is *parity unpinned* (only its inputs are).
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

LOG_2PI = float(np.log(2.0 * np.pi))


# --------------------------------------------------------------------------
# A1  ensemble reduction  (eks/ensemble_kalman.py:4-57)
# --------------------------------------------------------------------------
def ensemble_array(stack: np.ndarray, mode: str = "median"):
    """Median (or mean) and variance-of-the-mean over the member axis.

    ``stack`` is (E, T, n).  Follows eks/ensemble_kalman.py:34-46: the
    average is ``np.median`` / ``np.mean`` over members and the variance is
    ``np.var(ddof=0) / E`` in *both* modes (quirk 3).
    """
    if mode == "median":
        reduce = np.median
    elif mode == "mean":
        reduce = np.mean
    else:  # eks/ensemble_kalman.py:39
        raise ValueError(f"{mode} averaging not supported")
    stack = np.asarray(stack, dtype=np.float64)
    n_members = stack.shape[0]
    # reduce along a contiguous trailing axis, as the reference does on its
    # (T, E) per-key stacks (eks/ensemble_kalman.py:44-46)
    per_key = np.moveaxis(stack, 0, -1)  # (T, n, E)
    avg = reduce(per_key, axis=-1)
    var = np.var(per_key, axis=-1) / n_members
    return avg, var


def ensemble(markers_list, keys, mode: str = "median"):
    """DataFrame-level restatement of eks/ensemble_kalman.py:4-57.

    Returns the same 6-tuple: preds (T,n), vars (T,n), stacks (E,T,n), and
    the three dictionaries (key->avg, key->var, member->key->column).
    """
    stack = np.stack(
        [np.stack([np.asarray(df[k], dtype=np.float64) for k in keys], axis=1)
         for df in markers_list]
    )  # (E, T, n)
    preds, var = ensemble_array(stack, mode)
    avg_d = {k: preds[:, j] for j, k in enumerate(keys)}
    var_d = {k: var[:, j] for j, k in enumerate(keys)}
    stack_d = defaultdict(dict)
    for e in range(stack.shape[0]):
        for j, k in enumerate(keys):
            stack_d[e][k] = stack[e, :, j]
    return preds, var, stack, avg_d, var_d, stack_d


# --------------------------------------------------------------------------
# A2/A3  forward filter  (eks/ensemble_kalman.py:59-117)
# --------------------------------------------------------------------------
def kalman_dot(array, V, C, R):
    """``V C^T (R + C V C^T)^{-1} array`` with a dense LU solve.

    eks/ensemble_kalman.py:110-117 (LAPACK gesv through ``np.linalg.solve``).
    """
    innov_cov = R + np.dot(C, np.dot(V, C.T))
    return np.dot(V, np.dot(C.T, np.linalg.solve(innov_cov, array)))


def filtering_pass(y, m0, S0, C, R, A, Q, ensemble_vars):
    """Forward Kalman recursion with R_t = diag(ensemble_vars[t]).

    eks/ensemble_kalman.py:59-107.  Quirks kept: ``R``'s diagonal is
    overwritten in place every step (:88-89, :99-100), so the caller's R ends
    holding ``ensemble_vars[T-1]``; ``S[t]`` holds the covariance predicted
    *for* step t+1 (:101), and ``S[T-1]`` is never written (stays 0).
    """
    n_obs = ensemble_vars.shape[1]
    T = y.shape[0]
    r = m0.shape[0]
    mf = np.zeros((T, r))
    Vf = np.zeros((T, r, r))
    S = np.zeros((T, r, r))
    for i in range(n_obs):
        R[i, i] = ensemble_vars[0, i]
    mf[0] = m0 + kalman_dot(y[0] - np.dot(C, m0), S0, C, R)
    Vf[0] = S0 - kalman_dot(np.dot(C, S0), S0, C, R)
    S[0] = S0
    At = A.T
    for t in range(1, T):
        ev_t = ensemble_vars[t]
        for i in range(n_obs):
            R[i, i] = ev_t[i]
        prior_cov = np.dot(A, np.dot(Vf[t - 1], At)) + Q
        S[t - 1] = prior_cov
        prior_mean = np.dot(A, mf[t - 1])
        mf[t] = prior_mean + kalman_dot(y[t] - np.dot(C, prior_mean), prior_cov, C, R)
        Vf[t] = prior_cov - kalman_dot(np.dot(C, prior_cov), prior_cov, C, R)
    return mf, Vf, S


# --------------------------------------------------------------------------
# A4  RTS backward pass  (eks/ensemble_kalman.py:120-164)
# --------------------------------------------------------------------------
def smooth_backward(y, mf, Vf, S, A, Q=None, C=None):
    """Rauch-Tung-Striebel recursion.  ``Q`` and ``C`` are accepted and unused,
    and ``y`` only supplies T, as in eks/ensemble_kalman.py:146-162."""
    T = y.shape[0]
    r = mf.shape[1]
    ms = np.zeros((T, r))
    Vs = np.zeros((T, r, r))
    CV = np.zeros((max(T - 1, 0), r, r))
    ms[T - 1] = mf[T - 1]
    Vs[T - 1] = Vf[T - 1]
    for t in range(T - 2, -1, -1):
        gain = np.linalg.solve(S[t], np.dot(A, Vf[t])).T  # :158
        Vs[t] = Vf[t] + np.dot(gain, np.dot(Vs[t + 1] - S[t], gain.T))  # :160
        ms[t] = mf[t] + np.dot(gain, ms[t + 1] - np.dot(A, mf[t]))  # :161
        CV[t] = np.dot(Vs[t + 1], gain.T)  # :162
    return ms, Vs, CV


# --------------------------------------------------------------------------
# A5  negative log-likelihood  (build definition)
# --------------------------------------------------------------------------
def compute_nll(y, m0, S0, C, A, Q, ensemble_vars):
    """Gaussian innovation NLL of the filter, built from the terms of
    eks/ensemble_kalman.py:94, :102, :112:

        e_0 = y_0 - C m0,           Sigma_0 = R_0 + C S0 C^T
        e_t = y_t - C A mf[t-1],    Sigma_t = R_t + C S[t-1] C^T
        NLL = 1/2 sum_t [ n log 2pi + log det Sigma_t + e_t^T Sigma_t^-1 e_t ]

    Parity unpinned: the reference computes no likelihood.
    """
    mf, Vf, _ = filtering_pass(y, m0, S0, C, np.eye(C.shape[0]), A, Q, ensemble_vars)
    T, n = y.shape
    # predicted covariances for every step (S0 first, then A Vf A^T + Q)
    total = 0.0
    R = np.zeros((n, n))
    diag = np.arange(n)
    prior_m = m0
    prior_P = S0
    for t in range(T):
        if t > 0:
            prior_m = A @ mf[t - 1]
            prior_P = A @ Vf[t - 1] @ A.T + Q
        R[diag, diag] = ensemble_vars[t]
        sig = R + C @ prior_P @ C.T
        e = y[t] - C @ prior_m
        _, logdet = np.linalg.slogdet(sig)
        total += 0.5 * (n * LOG_2PI + logdet + e @ np.linalg.solve(sig, e))
    return float(total)


# --------------------------------------------------------------------------
# A6  single-view parameterisation  (build definition)
# --------------------------------------------------------------------------
def good_frames(ev: np.ndarray, quantile_keep: float) -> np.ndarray:
    """Frames whose max ensemble variance is <= the q-th percentile.

    eks/multiview_pca_smoother.py:685-688 (np.percentile, linear).
    """
    max_vars = np.max(ev, axis=1)
    return np.where(max_vars <= np.percentile(max_vars, quantile_keep))[0]


def singleview_params(preds, ev, smooth_param, quantile_keep):
    """m0, S0, A, Q, C, offsets for one keypoint, per SURVEY.md §8 A6
    (template: eks/multiview_pca_smoother.py:684-731 without the PCA)."""
    good = good_frames(ev, quantile_keep)
    means = preds[good].mean(axis=0)
    yc = preds - means
    good_y = yc[good]
    m0 = np.zeros(2)
    S0 = np.diag(np.var(good_y, axis=0))
    A = np.eye(2)
    C = np.eye(2)
    Q = smooth_param * np.cov((good_y[1:] - good_y[:-1]).T)
    return dict(m0=m0, S0=S0, A=A, Q=Q, C=C, means=means, y=yc, good=good)


def singleview_smooth(stack, smooth_param, quantile_keep, mode="median"):
    """Whole single-view path for one keypoint: (E,T,2) -> smoothed (T,2)."""
    preds, ev = ensemble_array(stack, mode)
    p = singleview_params(preds, ev, smooth_param, quantile_keep)
    R = np.eye(2)
    mf, Vf, S = filtering_pass(p["y"], p["m0"], p["S0"], p["C"], R, p["A"], p["Q"], ev)
    ms, Vs, _ = smooth_backward(p["y"], mf, Vf, S, p["A"])
    return ms @ p["C"].T + p["means"], p, (mf, Vf, S, ms, Vs)


# --------------------------------------------------------------------------
# A7  multi-camera PCA smoother  (eks/multiview_pca_smoother.py:611-767)
# --------------------------------------------------------------------------
def pca_components(X: np.ndarray, n_comps: int):
    """Principal axes of X (rows = samples), as sklearn's 'covariance_eigh'
    solver finds them (eigen-decomposition of the sample covariance).  The
    sign of each axis is arbitrary; outputs are invariant to it because S0 is
    diagonal."""
    Xc = X - X.mean(axis=0)
    cov = Xc.T @ Xc / (X.shape[0] - 1)
    w, v = np.linalg.eigh(cov)
    order = np.argsort(w)[::-1][:n_comps]
    return v[:, order].T, X.mean(axis=0)


def multicam_params(cam_preds, cam_vars, smooth_param, quantile_keep):
    """cam_preds/cam_vars: (T, 2V) hstacked per-camera ensemble outputs.

    eks/multiview_pca_smoother.py:684-731."""
    good = good_frames(cam_vars, quantile_keep)
    means = cam_preds[good].mean(axis=0)
    y = cam_preds - means
    comps, mean_ = pca_components(y[good], 3)
    pcs = (y - mean_) @ comps.T
    good_pcs = pcs[good]
    m0 = np.zeros(3)
    S0 = np.diag(np.var(good_pcs, axis=0))
    A = np.eye(3)
    Q = smooth_param * np.cov((good_pcs[1:] - good_pcs[:-1]).T)
    C = comps.T
    return dict(m0=m0, S0=S0, A=A, Q=Q, C=C, means=means, y=y, good=good)


def multicam_smooth(cam_stacks, smooth_param, quantile_keep, mode="median"):
    """cam_stacks: list over cameras of (E, T, 2) arrays -> (T, 2V) output
    (camera-major x,y columns), eks/multiview_pca_smoother.py:641-765."""
    preds, ev = [], []
    for st in cam_stacks:
        p_, v_ = ensemble_array(st, mode)
        preds.append(p_)
        ev.append(v_)
    preds = np.hstack(preds)
    ev = np.hstack(ev)
    p = multicam_params(preds, ev, smooth_param, quantile_keep)
    R = np.eye(preds.shape[1])  # placeholder, :731 (eye of 2V)
    mf, Vf, S = filtering_pass(p["y"], p["m0"], p["S0"], p["C"], R, p["A"], p["Q"], ev)
    ms, Vs, _ = smooth_backward(p["y"], mf, Vf, S, p["A"])
    return ms @ p["C"].T + p["means"], p, ev


# --------------------------------------------------------------------------
# A8  IBL pupil smoother  (eks/pupil_smoother.py:82-223)
# --------------------------------------------------------------------------
PUPIL_KEYS = ['pupil_top_r_x', 'pupil_top_r_y', 'pupil_bottom_r_x', 'pupil_bottom_r_y',
              'pupil_right_r_x', 'pupil_right_r_y', 'pupil_left_r_x', 'pupil_left_r_y']
PUPIL_C = np.array([[0, 1, 0], [-.5, 0, 1], [0, 1, 0], [.5, 0, 1],
                    [.5, 1, 0], [0, 0, 1], [-.5, 1, 0], [0, 0, 1]], dtype=np.float64)


def pupil_center(cols: dict) -> np.ndarray:
    """eks/pupil_smoother.py:14-39 (nanmedian/median combinations)."""
    t = np.stack([cols['pupil_top_r_x'], cols['pupil_top_r_y']], axis=1)
    b = np.stack([cols['pupil_bottom_r_x'], cols['pupil_bottom_r_y']], axis=1)
    l_ = np.stack([cols['pupil_left_r_x'], cols['pupil_left_r_y']], axis=1)
    r_ = np.stack([cols['pupil_right_r_x'], cols['pupil_right_r_y']], axis=1)
    cx1 = np.nanmedian(np.stack([t[:, 0], b[:, 0]], axis=1), axis=1)
    cx2 = np.median(np.stack([r_[:, 0], l_[:, 0]], axis=1), axis=1)
    cy1 = np.median(np.stack([t[:, 1], b[:, 1]], axis=1), axis=1)
    cy2 = np.nanmedian(np.stack([r_[:, 1], l_[:, 1]], axis=1), axis=1)
    cx = np.nanmedian(np.stack([cx1, cx2], axis=1), axis=1)
    cy = np.nanmedian(np.stack([cy1, cy2], axis=1), axis=1)
    return np.stack([cx, cy], axis=1)


def pupil_diameter(cols: dict) -> np.ndarray:
    """eks/pupil_smoother.py:42-68: nanmedian of two direct and four
    circle-assumption (x sqrt 2) diameter estimates."""
    pts = {p: np.stack([cols[f'pupil_{p}_r_x'], cols[f'pupil_{p}_r_y']])
           for p in ('top', 'bottom', 'left', 'right')}
    est = [np.linalg.norm(pts['top'] - pts['bottom'], axis=0),
           np.linalg.norm(pts['left'] - pts['right'], axis=0)]
    for a, b in (('top', 'left'), ('top', 'right'), ('bottom', 'left'), ('bottom', 'right')):
        est.append(np.linalg.norm(pts[a] - pts[b], axis=0) * 2 ** 0.5)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", category=RuntimeWarning)
        return np.nanmedian(est, axis=0)


def pupil_params(preds, A):
    """eks/pupil_smoother.py:109-172."""
    cols = {k: preds[:, j] for j, k in enumerate(PUPIL_KEYS)}
    centre = pupil_center(cols)
    diam = pupil_diameter(cols)
    mx = np.mean(centre[:, 0])
    my = np.mean(centre[:, 1])
    cx = centre[:, 0] - mx
    cy = centre[:, 1] - my
    m0 = np.array([np.mean(diam), 0.0, 0.0])
    var_d, var_x, var_y = np.var(diam), np.var(cx), np.var(cy)
    S0 = np.diag([var_d, var_x, var_y])
    Q = np.diag([var_d * (1 - A[0, 0] ** 2), var_x * (1 - A[1, 1] ** 2),
                 var_y * (1 - A[2, 2] ** 2)])
    offs = np.array([mx if j % 2 == 0 else my for j in range(8)])
    return dict(m0=m0, S0=S0, A=np.asarray(A, dtype=np.float64), Q=Q, C=PUPIL_C.copy(),
                means=offs, y=preds - offs, mx=mx, my=my)


def pupil_smooth(stack, A, mode="median"):
    """stack (E, T, 8) in PUPIL_KEYS order -> (markers (T,8) in key order,
    latents (T,3) = diameter, com_x + mx, com_y + my)."""
    preds, ev = ensemble_array(stack, mode)
    p = pupil_params(preds, A)
    R = np.eye(8)
    mf, Vf, S = filtering_pass(p["y"], p["m0"], p["S0"], p["C"], R, p["A"], p["Q"], ev)
    ms, Vs, _ = smooth_backward(p["y"], mf, Vf, S, p["A"])
    markers = ms @ p["C"].T + p["means"]
    latents = np.stack([ms[:, 0], ms[:, 1] + p["mx"], ms[:, 2] + p["my"]], axis=1)
    return markers, latents, p, ev


# --------------------------------------------------------------------------
# F3  Newton "opti" forward filter  (eks/newton_eks.py:115-148)
# --------------------------------------------------------------------------
def kalman_newton_recursive(y, mu0, S0, A, B, ensemble_vars, E, max_iter=1):
    """Information-form forward filter of eks/newton_eks.py:115-148 with its
    quirks: q[0] = mu0 with no measurement update, P starts as inv(S0) (used
    as a covariance), P carries over between iterations, and q is updated in
    place (the reference's ``qnew = q`` alias), so every iteration's loss is 0.
    For T == 1 the trailing step reads q[T-2] = q[-1] = q[0]."""
    T = y.shape[0]
    q = np.zeros((T, mu0.shape[0]))
    q[0] = mu0
    P = np.linalg.inv(S0)
    loss = np.zeros(max_iter)
    for it in range(max_iter):
        for t in range(1, T):
            invD = np.linalg.inv(np.diag(ensemble_vars[t]))
            P = np.linalg.inv(np.linalg.inv(E + A @ P @ A.T) + B.T @ invD @ B)
            q[t] = A @ q[t - 1] - P @ B.T @ invD @ (B @ A @ q[t - 1] - y[t])
        if T == 1:  # the reference's separate last step with q[T-2] == q[-1]
            invD = np.linalg.inv(np.diag(ensemble_vars[0]))
            P = np.linalg.inv(np.linalg.inv(E + A @ P @ A.T) + B.T @ invD @ B)
            q[0] = A @ q[0] - P @ B.T @ invD @ (B @ A @ q[0] - y[0])
        loss[it] = 0.0
    if max_iter == 1:
        return q
    return q, loss


def multicam_opti_smooth(cam_stacks, smooth_param, quantile_keep, mode="median"):
    """eks_opti_smoother_multi_cam (eks/multiview_pca_smoother.py:777-933):
    the multicam model fit, then the Newton filter (no backward pass)."""
    preds, ev = [], []
    for st in cam_stacks:
        p_, v_ = ensemble_array(st, mode)
        preds.append(p_)
        ev.append(v_)
    preds = np.hstack(preds)
    ev = np.hstack(ev)
    p = multicam_params(preds, ev, smooth_param, quantile_keep)
    q = kalman_newton_recursive(p["y"], p["m0"], p["S0"], p["A"], p["C"], ev, p["Q"])
    return q @ p["C"].T + p["means"], p, q


def pupil_opti_smooth(stack, mode="median"):
    """eks_opti_smoother_pupil (eks/pupil_smoother.py:227-320) as intended:
    the pupil model with the hard-coded A = 0.99 I (:260), Newton filter,
    latents = (diameter, com_x + mx, com_y + my) and markers = C q + offsets.
    (The reference's plot=False branch references an undefined q; the committed
    data/misc/pupil-test/opti_eks_latents.csv is this computation.)"""
    preds, ev = ensemble_array(stack, mode)
    p = pupil_params(preds, np.diag([0.99, 0.99, 0.99]))
    q = kalman_newton_recursive(p["y"], p["m0"], p["S0"], p["A"], p["C"], ev, p["Q"])
    markers = q @ p["C"].T + p["means"]
    latents = np.stack([q[:, 0], q[:, 1] + p["mx"], q[:, 2] + p["my"]], axis=1)
    return markers, latents, p, ev


# --------------------------------------------------------------------------
# F4  asynchronous two-camera paw smoother
#     (eks/multiview_pca_smoother.py:34-322 standard, :325-574 opti)
# --------------------------------------------------------------------------
PAW_IMG_WIDTH = 128


def paw_async_select(tl, tr):
    """Left-camera frames the reference keeps (:86-90): in order, skipping
    ts < tr[0], stopping at the first ts > tr[-1]."""
    keep = []
    for i, ts in enumerate(tl):
        if ts > tr[-1]:
            break
        if ts < tr[0]:
            continue
        keep.append(i)
    return np.asarray(keep, dtype=np.int64)


def paw_async_smooth(left_np, right_np, tl, tr, smooth_param, quantile_keep, opti=False):
    """left_np / right_np: (E, T_cam, >= 5) member arrays (x, y, likelihood of
    paw 1 then paw 2, as convert_lp_dlc orders them).  Returns (left (T, 4),
    right (T, 4)) smoothed (x, y) pairs in the reference's output order:
    left = (paw 1 x, y, paw 2 x, y) in the left view; right = (paw 2 x, y,
    paw 1 x, y) in the right view, x flipped back (:300-320)."""
    sel = paw_async_select(tl, tr)
    cols = [0, 1, 3, 4]
    E = left_np.shape[0]
    Lc = np.stack([left_np[e][sel][:, cols] for e in range(E)])            # (E, T, 4)
    Rc = np.stack([np.stack([np.interp(tl[sel], tr, right_np[e][:, j]) for j in cols], 1)
                   for e in range(E)])
    Rc[:, :, 0] = PAW_IMG_WIDTH - Rc[:, :, 0]
    Rc[:, :, 2] = PAW_IMG_WIDTH - Rc[:, :, 2]
    lp, lv = ensemble_array(Lc)
    rp, rv = ensemble_array(Rc)
    worst = np.max(np.hstack([lv, rv]), 1)
    good = np.where(worst <= np.percentile(worst, quantile_keep))[0]
    stacked = np.empty((2 * len(good), 4))
    stacked[0::2] = np.hstack([lp[good][:, :2], rp[good][:, :2]])
    stacked[1::2] = np.hstack([lp[good][:, 2:4], rp[good][:, 2:4]])
    means = stacked.mean(axis=0)
    comps, mean_ = pca_components(stacked - means, 3)
    C = comps.T
    paws = {"left": (np.hstack([lp[:, :2], rp[:, :2]]), np.hstack([lv[:, :2], rv[:, :2]])),
            "right": (np.hstack([lp[:, 2:4], rp[:, 2:4]]), np.hstack([lv[:, 2:4], rv[:, 2:4]]))}
    outs = {}
    for paw, (pred, var) in paws.items():
        y = pred - means
        good_pcs = ((y - mean_) @ comps.T)[good]
        S0 = np.diag(np.var(good_pcs, axis=0))
        Q = smooth_param * np.cov((good_pcs[1:] - good_pcs[:-1]).T)
        if opti:
            q = kalman_newton_recursive(y, np.zeros(3), S0, np.eye(3), C, var, Q)
        else:
            R = np.eye(4)
            mf, Vf, S = filtering_pass(y, np.zeros(3), S0, C, R, np.eye(3), Q, var)
            q, _, _ = smooth_backward(y, mf, Vf, S, np.eye(3))
        outs[paw] = q @ C.T + means
    left = np.stack([outs["left"][:, 0], outs["left"][:, 1],
                     outs["right"][:, 0], outs["right"][:, 1]], 1)
    right = np.stack([PAW_IMG_WIDTH - outs["right"][:, 2], outs["right"][:, 3],
                      PAW_IMG_WIDTH - outs["left"][:, 2], outs["left"][:, 3]], 1)
    return left, right
