"""Per-keypoint entry points, API-compatible with the reference wrappers.

    ensemble_kalman_smoother_multi_cam   eks/multiview_pca_smoother.py:611-767
    ensemble_kalman_smoother_pupil       eks/pupil_smoother.py:82-223
    ensemble_kalman_smoother_single_view build definition
    eks_opti_smoother_multi_cam          eks/multiview_pca_smoother.py:777-933
    eks_opti_smoother_pupil              eks/pupil_smoother.py:227-320

Flow for one keypoint: member DataFrames -> (E, T, n) array -> GPU ensemble
(eks_ensemble, written as the y / ev hand-off planes) -> host model fit
(eks_amd.fit, on the planes' host copies) -> GPU fused smoother from the
planes (eks_smooth: forward, backward, projection) -> DataFrames in the
reference's output format.  The members are uploaded and reduced once; no
step of the smoother runs on the CPU.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from . import _lib, batch, core, fit
from .newton_eks import kalman_newton_recursive, newton_filter_batch
from .utils import TRACKER, make_dlc_pandas_index


def _run_fused(stack: np.ndarray, model: dict, mode: str = "median", want_ms=False,
               want_nll=False, yev=None):
    """stack (E, T, n) float64 host array + model -> out (T, n), ms, nll.
    With ``yev`` (core.ensemble_handoff's planes of the same stack) the
    smoother reads the planes instead of uploading and reducing the members
    again (every algorithm, the runtime-n kernels included)."""
    torch = _lib.require_gpu()
    E, T, n = stack.shape
    r = len(model["m0"])
    if yev is not None:
        obs = yev
    else:
        obs = torch.from_numpy(np.ascontiguousarray(stack, dtype=np.float64)).to("cuda")
        obs = obs.permute(1, 0, 2).unsqueeze(0)  # (1, T, E, n) view, no copy
    params = batch.pack_params(model["m0"], model["S0"], model["A"], model["Q"], model["C"],
                               model["offset"])
    res = batch.smooth(obs, params, n=n, r=r, mode=mode, want_ms=want_ms, want_nll=want_nll,
                       flags=batch.model_flags(model["A"], model["C"], model["Q"]), check=True)
    out = res["out"][0].cpu().numpy()
    ms = res["ms"][0].cpu().numpy() if want_ms else None
    nll = float(res["nll"][0].item()) if want_nll else None
    return out, ms, nll


def ensemble_kalman_smoother_multi_cam(markers_list_cameras, keypoint_ensemble, smooth_param,
                                       quantile_keep_pca, camera_names):
    """Multi-view PCA smoother for one keypoint (eks/multiview_pca_smoother.py:611-767).

    markers_list_cameras[camera][model] is a DataFrame whose first two
    columns are that camera's x and y predictions.  Returns
    {f'{camera}_df': DataFrame} with (scorer, keypoint, x/y/likelihood)
    columns; likelihood is NaN as in the reference."""
    V = len(camera_names)
    if V < 2:
        raise ValueError("ensemble_kalman_smoother_multi_cam needs at least two cameras "
                         "(the reference's 3-component PCA needs >= 3 columns); use "
                         "ensemble_kalman_smoother_single_view for one view")
    n_models = len(markers_list_cameras[0])
    cols = [np.stack([np.asarray(markers_list_cameras[c][e].to_numpy()[:, :2], dtype=np.float64)
                      for e in range(n_models)]) for c in range(V)]  # V x (E, T, 2)
    stack = np.concatenate(cols, axis=2)  # (E, T, 2V), camera-major columns
    yev, preds, ev = core.ensemble_handoff(stack)
    model = fit.multicam_model(preds, ev, smooth_param, quantile_keep_pca)
    out, _, _ = _run_fused(stack, model, yev=yev)
    pdindex = make_dlc_pandas_index([keypoint_ensemble])
    dfs = {}
    nan = np.full(out.shape[0], np.nan)
    for c, cam in enumerate(camera_names):
        arr = np.stack([out[:, 2 * c], out[:, 2 * c + 1], nan], axis=1)
        dfs[cam + "_df"] = pd.DataFrame(arr, columns=pdindex)
    return dfs


def ensemble_kalman_smoother_pupil(markers_list, keypoint_names, tracker_name,
                                   state_transition_matrix):
    """IBL pupil smoother (eks/pupil_smoother.py:82-223).

    Returns {'markers_df': smoothed keypoints in the order top, right, bottom,
    left (NaN likelihood), 'latents_df': diameter, com_x, com_y}."""
    stack = np.stack([np.stack([np.asarray(df[k], dtype=np.float64) for k in fit.PUPIL_KEYS], 1)
                      for df in markers_list])  # (E, T, 8)
    yev, preds, _ = core.ensemble_handoff(stack)
    model = fit.pupil_model(preds, state_transition_matrix)
    out, ms, _ = _run_fused(stack, model, want_ms=True, yev=yev)
    by_key = {k: out[:, j] for j, k in enumerate(fit.PUPIL_KEYS)}
    nan = np.full(out.shape[0], np.nan)
    cols = []
    for kp in ('top', 'right', 'bottom', 'left'):  # output order of :199-203
        cols += [by_key[f'pupil_{kp}_r_x'], by_key[f'pupil_{kp}_r_y'], nan]
    markers_df = pd.DataFrame(np.stack(cols, 1), columns=make_dlc_pandas_index(keypoint_names))
    lat = np.stack([ms[:, 0], ms[:, 1] + model["mx"], ms[:, 2] + model["my"]], 1)
    idx = pd.MultiIndex.from_arrays([[tracker_name] * 3, ['diameter', 'com_x', 'com_y']],
                                    names=('scorer', 'latent'))
    return {'markers_df': markers_df, 'latents_df': pd.DataFrame(lat, columns=idx)}


def pupil_smoothing_sweep(markers_list, keypoint_names, tracker_name, diameter_s_grid,
                          com_s_grid):
    """The pupil smoother with its smoothing parameters chosen by likelihood.

    Every (diameter_s, com_s) pair of the grid defines a model
    (A = diag(d, c, c), Q = var (1 - A^2): eks/pupil_smoother.py:140-147);
    all candidates are scored in ONE filter-only batched call (the member
    predictions are shared, batch stride 0) by their innovation NLL, and the
    argmin is smoothed.  Returns ensemble_kalman_smoother_pupil's dict plus
    'nll' (len(diameter_s_grid), len(com_s_grid)) and 'best' (d, c).
    (The reference has no NLL loop: SURVEY.md §0; this is the build's.)"""
    torch = _lib.require_gpu()
    stack = np.stack([np.stack([np.asarray(df[k], dtype=np.float64) for k in fit.PUPIL_KEYS], 1)
                      for df in markers_list])  # (E, T, 8)
    E, T, n = stack.shape
    preds, _ = core.ensemble_array(stack)
    grid = [(d, c) for d in diameter_s_grid for c in com_s_grid]
    models = [fit.pupil_model(preds, np.diag([d, c, c])) for d, c in grid]
    stackp = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stackp("m0"), stackp("S0"), stackp("A"), stackp("Q"),
                               stackp("C"), stackp("offset"))
    obs = torch.from_numpy(np.ascontiguousarray(stack)).to("cuda").permute(1, 0, 2).unsqueeze(0)
    flags = batch.model_flags(stackp("A"), stackp("C"), stackp("Q"))
    scores = batch.nll(obs.expand(len(grid), -1, -1, -1), params, n=n, r=3,
                       flags=flags).cpu().numpy()
    best = grid[int(np.argmin(scores))]
    res = ensemble_kalman_smoother_pupil(markers_list, keypoint_names, tracker_name,
                                         np.diag([best[0], best[1], best[1]]))
    res["nll"] = scores.reshape(len(diameter_s_grid), len(com_s_grid))
    res["best"] = best
    return res


def ensemble_kalman_smoother_single_view(markers_list, keypoint_ensemble, smooth_param,
                                         quantile_keep_pca=25, ensembling_mode="median"):
    """Single-view EKS for one keypoint (the reference
    snapshot has no single-view smoother).

    markers_list: E DataFrames with '{keypoint}_x' / '{keypoint}_y' columns.
    Model: C = A = I2, m0 = 0, S0 = diag(var), Q = s cov(diff) over the
    low-variance frames, offset = their mean.  Returns {'markers_df',
    'nll'} with the reference's output format."""
    keys = [f"{keypoint_ensemble}_x", f"{keypoint_ensemble}_y"]
    stack = np.stack([np.stack([np.asarray(df[k], dtype=np.float64) for k in keys], 1)
                      for df in markers_list])  # (E, T, 2)
    yev, preds, ev = core.ensemble_handoff(stack, ensembling_mode)
    model = fit.singleview_model(preds, ev, smooth_param, quantile_keep_pca)
    out, _, nll = _run_fused(stack, model, mode=ensembling_mode, want_nll=True, yev=yev)
    nan = np.full(out.shape[0], np.nan)
    df = pd.DataFrame(np.stack([out[:, 0], out[:, 1], nan], 1),
                      columns=make_dlc_pandas_index([keypoint_ensemble]))
    return {'markers_df': df, 'nll': nll}




def _camera_dfs(out, keypoint_ensemble, camera_names):
    pdindex = make_dlc_pandas_index([keypoint_ensemble])
    nan = np.full(out.shape[0], np.nan)
    return {cam + "_df": pd.DataFrame(np.stack([out[:, 2 * c], out[:, 2 * c + 1], nan], axis=1),
                                      columns=pdindex)
            for c, cam in enumerate(camera_names)}


def eks_opti_smoother_multi_cam(markers_list_cameras, keypoint_ensemble, smooth_param,
                                quantile_keep_pca, camera_names, plot=False):
    """Multi-view PCA model + Newton forward filter, no backward pass
    (eks/multiview_pca_smoother.py:777-933): the model fit of
    ensemble_kalman_smoother_multi_cam, then kalman_newton_recursive with
    B = PCA axes, E = smooth_param * cov(diff(pcs)), output B q + means.
    ``plot`` is accepted for signature compatibility; the reference's plot
    branch reads a developer-local file, so nothing is plotted."""
    V = len(camera_names)
    if V < 2:
        raise ValueError("eks_opti_smoother_multi_cam needs at least two cameras")
    n_models = len(markers_list_cameras[0])
    cols = [np.stack([np.asarray(markers_list_cameras[c][e].to_numpy()[:, :2], dtype=np.float64)
                      for e in range(n_models)]) for c in range(V)]
    stack = np.concatenate(cols, axis=2)
    preds, ev = core.ensemble_array(stack)
    model = fit.multicam_model(preds, ev, smooth_param, quantile_keep_pca)
    q = kalman_newton_recursive(preds - model["offset"], model["m0"], model["S0"], model["A"],
                                model["C"], ev, model["Q"])
    out = q @ model["C"].T + model["offset"]
    return _camera_dfs(out, keypoint_ensemble, camera_names)


def eks_opti_smoother_pupil(markers_list, keypoint_names, tracker_name, state_transition_matrix,
                            plot=False):
    """IBL pupil model + Newton forward filter (eks/pupil_smoother.py:227-320).

    As in the reference, the transition matrix is fixed at A = 0.99 I (:260)
    and ``state_transition_matrix`` is ignored.  The reference's plot=False
    branch then uses an undefined variable; this returns what its plot=True
    branch and the committed data/misc/pupil-test/opti_eks_latents.csv hold:
    markers_df (C q + offsets, order top, right, bottom, left, NaN likelihood)
    and latents_df (diameter, com_x, com_y)."""
    stack = np.stack([np.stack([np.asarray(df[k], dtype=np.float64) for k in fit.PUPIL_KEYS], 1)
                      for df in markers_list])
    preds, ev = core.ensemble_array(stack)
    model = fit.pupil_model(preds, np.diag([0.99, 0.99, 0.99]))
    q = kalman_newton_recursive(preds - model["offset"], model["m0"], model["S0"], model["A"],
                                model["C"], ev, model["Q"])
    out = q @ model["C"].T + model["offset"]
    by_key = {k: out[:, j] for j, k in enumerate(fit.PUPIL_KEYS)}
    nan = np.full(out.shape[0], np.nan)
    cols = []
    for kp in ('top', 'right', 'bottom', 'left'):
        cols += [by_key[f'pupil_{kp}_r_x'], by_key[f'pupil_{kp}_r_y'], nan]
    markers_df = pd.DataFrame(np.stack(cols, 1), columns=make_dlc_pandas_index(keypoint_names))
    lat = np.stack([q[:, 0], q[:, 1] + model["mx"], q[:, 2] + model["my"]], 1)
    idx = pd.MultiIndex.from_arrays([[tracker_name] * 3, ['diameter', 'com_x', 'com_y']],
                                    names=('scorer', 'latent'))
    return {'markers_df': markers_df, 'latents_df': pd.DataFrame(lat, columns=idx)}


def ensemble_stacks(stacks, mode: str = "median"):
    """(K, E, T, n) member array (numpy or CUDA tensor) of K trajectories ->
    (members on the device, preds, vars (K, T, n)) CUDA float64, one
    eks_ensemble launch."""
    torch = _lib.require_gpu()
    if mode not in ("median", "mean"):
        raise ValueError(f"{mode} averaging not supported")
    K, E, T, n = stacks.shape
    if torch.is_tensor(stacks):
        d = stacks.to(device="cuda", dtype=torch.float64).contiguous()
    else:
        d = torch.from_numpy(np.ascontiguousarray(stacks, dtype=np.float64)).to("cuda")
    preds = torch.empty((K, T, n), dtype=torch.float64, device="cuda")
    var = torch.empty_like(preds)
    lib = _lib.load()
    _lib.check(lib.eks_ensemble(d.data_ptr(), _lib.EKS_F64, K, T, E, n, E * T * n, n, T * n, 1,
                                _lib.EKS_MEDIAN if mode == "median" else _lib.EKS_MEAN,
                                preds.data_ptr(), var.data_ptr(), _lib.stream_ptr()),
               "eks_ensemble")
    return d, preds, var


def multi_cam_batch(stacks, smooth_param, quantile_keep_pca, version: str = "standard"):
    """All keypoints of a multi-camera dataset in one launch each for the
    ensemble and the smoother (the reference loops keypoints one call at a
    time: scripts/multicam_example.py:106-150).

    stacks (K, E, T, 2V) camera-major (x, y) columns per keypoint.  The
    per-keypoint model fit is ensemble_kalman_smoother_multi_cam's
    (eks/multiview_pca_smoother.py:684-731); version "standard" fits every
    keypoint's model on the device (eks_fit, 1-8 cameras) and runs the fused
    RTS smoother (eks_smooth) on the fit's ensemble hand-off planes, "opti"
    fits on the host and runs the Newton filter (eks_newton_filter,
    :777-933).  Returns out (K, T, 2V) float64 numpy."""
    torch = _lib.require_gpu()
    stacks = np.asarray(stacks, dtype=np.float64)
    K, E, T, n = stacks.shape
    if n < 4:
        raise ValueError("multi-camera smoothing needs at least two cameras")
    if version != "opti" and n % 2 == 0 and n <= 16:
        obs = torch.from_numpy(np.ascontiguousarray(stacks)).to("cuda").permute(0, 2, 1, 3)
        params, _, yev = batch.fit(obs, kind="multicam", n=n, r=3, smooth_param=smooth_param,
                                   quantile_keep=quantile_keep_pca, keep_yev=True)
        res = batch.smooth(yev, params, n=n, r=3, flags=_lib.EKS_MODEL_A_IDENTITY, check=True)
        return res["out"].cpu().numpy()
    d, preds_d, ev_d = ensemble_stacks(stacks)
    preds, ev = preds_d.cpu().numpy(), ev_d.cpu().numpy()
    models = [fit.multicam_model(preds[k], ev[k], smooth_param, quantile_keep_pca)
              for k in range(K)]
    st = lambda key: np.stack([m[key] for m in models])  # noqa: E731
    if version == "opti":
        y = preds_d - torch.from_numpy(st("offset")).to("cuda")[:, None, :]
        q, status = newton_filter_batch(y, ev_d, st("m0"), st("S0"), st("A"), st("C"), st("Q"))
        if bool((status != 0).any()):
            raise np.linalg.LinAlgError("Singular matrix (kalman_newton_recursive)")
        q = q.cpu().numpy()
        return np.einsum("ktr,knr->ktn", q, st("C")) + st("offset")[:, None, :]
    params = batch.pack_params(st("m0"), st("S0"), st("A"), st("Q"), st("C"), st("offset"))
    obs = d.permute(0, 2, 1, 3)  # (K, T, E, n) view
    res = batch.smooth(obs, params, n=n, r=3, flags=batch.model_flags(st("A"), st("C")),
                       check=True)
    return res["out"].cpu().numpy()


__all__ = ["ensemble_kalman_smoother_multi_cam", "ensemble_kalman_smoother_pupil",
           "ensemble_kalman_smoother_single_view", "pupil_smoothing_sweep",
           "eks_opti_smoother_multi_cam", "eks_opti_smoother_pupil", "multi_cam_batch",
           "ensemble_stacks", "TRACKER"]


# --------------------------------------------------------------------------
# F4: asynchronous two-camera paw smoother
# --------------------------------------------------------------------------
PAW_IMG_WIDTH = 128


def interp1d_linear(x, y, xq):
    """np.interp / interp1d(kind='linear') of every column of y (n, C) at xq,
    on the GPU (eks_interp1d); bit-identical to numpy.  CUDA tensors in and
    out (float64)."""
    torch = _lib.require_gpu()
    x = torch.as_tensor(x, dtype=torch.float64, device="cuda").contiguous()
    xq = torch.as_tensor(xq, dtype=torch.float64, device="cuda").contiguous()
    y = torch.as_tensor(y, dtype=torch.float64, device="cuda")
    n, C = y.shape
    out = torch.empty((len(xq), C), dtype=torch.float64, device="cuda")
    status = torch.zeros(len(xq), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().eks_interp1d(x.data_ptr(), n, y.data_ptr(), C, y.stride(0),
                                        y.stride(1), xq.data_ptr(), len(xq), out.data_ptr(),
                                        out.stride(0), out.stride(1), status.data_ptr(),
                                        _lib.stream_ptr()), "eks_interp1d")
    if bool((status != 0).any()):
        raise ValueError("A value in x_new is outside the interpolation range.")
    return out


def _paw_async(markers_list_left_cam, markers_list_right_cam, timestamps_left_cam,
               timestamps_right_cam, keypoint_names, smooth_param, quantile_keep_pca, opti):
    torch = _lib.require_gpu()
    tl = np.asarray(timestamps_left_cam, dtype=np.float64)
    tr = np.asarray(timestamps_right_cam, dtype=np.float64)
    # left-camera frames inside the right camera's time span, in the
    # reference's loop order (:86-90): skip early frames, stop at the first late one
    late = np.flatnonzero(tl > tr[-1])
    stop = late[0] if len(late) else len(tl)
    sel = np.flatnonzero(tl[:stop] >= tr[0])
    cols = [0, 1, 3, 4]  # (x, y) of paw 1 and paw 2, likelihoods skipped
    E = len(markers_list_left_cam)
    left = np.stack([m.to_numpy()[sel][:, cols] for m in markers_list_left_cam])   # (E, T, 4)
    right_raw = np.stack([m.to_numpy()[:, cols] for m in markers_list_right_cam])  # (E, Tr, 4)
    T = len(sel)
    # right camera resampled at the kept left timestamps, x flipped (:92-94)
    rr = torch.from_numpy(np.ascontiguousarray(right_raw.transpose(1, 0, 2).reshape(len(tr), -1)))
    right = interp1d_linear(tr, rr.cuda(), tl[sel]).reshape(T, E, 4).permute(1, 0, 2).contiguous()
    right[:, :, 0] = PAW_IMG_WIDTH - right[:, :, 0]
    right[:, :, 2] = PAW_IMG_WIDTH - right[:, :, 2]
    cams = torch.stack([torch.from_numpy(left).cuda(), right])                    # (2, E, T, 4)
    _, preds_d, ev_d = ensemble_stacks(cams)
    preds, ev = preds_d.cpu().numpy(), ev_d.cpu().numpy()
    models, paw_stacks = fit.paw_async_models(preds, ev, smooth_param, quantile_keep_pca)
    st = lambda key: np.stack([m[key] for m in models])  # noqa: E731
    n = 4
    if opti:
        y = np.stack([models[k]["y"] for k in range(2)])
        v = np.stack([models[k]["ev"] for k in range(2)])
        q, status = newton_filter_batch(y, v, st("m0"), st("S0"), st("A"), st("C"), st("Q"))
        if bool((status != 0).any()):
            raise np.linalg.LinAlgError("Singular matrix (kalman_newton_recursive)")
        out = np.einsum("ktr,knr->ktn", q.cpu().numpy(), st("C")) + st("offset")[:, None, :]
    else:
        # per-paw member stacks (left view x, y | right view x, y): the fused
        # smoother ensembles them again, bit-identically
        obs = torch.stack([torch.cat([cams[0][:, :, 2 * k:2 * k + 2], cams[1][:, :, 2 * k:2 * k + 2]],
                                     dim=2) for k in range(2)])                   # (2, E, T, 4)
        params = batch.pack_params(st("m0"), st("S0"), st("A"), st("Q"), st("C"), st("offset"))
        res = batch.smooth(obs.permute(0, 2, 1, 3), params, n=n, r=3,
                           flags=_lib.EKS_MODEL_A_IDENTITY, check=True)
        out = res["out"].cpu().numpy()
    lp, rp = out[0], out[1]  # paw 1 / paw 2: (left x, y, right x, y)
    nan = np.full(T, np.nan)
    idx = make_dlc_pandas_index(keypoint_names)
    df_left = pd.DataFrame(np.stack([lp[:, 0], lp[:, 1], nan, rp[:, 0], rp[:, 1], nan], 1),
                           columns=idx)
    # right view: paws swapped back and x flipped to the LP convention (:309-320)
    df_right = pd.DataFrame(np.stack([PAW_IMG_WIDTH - rp[:, 2], rp[:, 3], nan,
                                      PAW_IMG_WIDTH - lp[:, 2], lp[:, 3], nan], 1), columns=idx)
    return {'left_df': df_left, 'right_df': df_right}


def ensemble_kalman_smoother_paw_asynchronous(
        markers_list_left_cam, markers_list_right_cam, timestamps_left_cam,
        timestamps_right_cam, keypoint_names, smooth_param, quantile_keep_pca):
    """Two asynchronous cameras, two paws (eks/multiview_pca_smoother.py:34-322):
    the right camera is resampled at the left camera's timestamps (GPU linear
    interpolation, eks_interp1d), one 3-D PCA subspace is fitted on both paws'
    good frames, and both paws are smoothed in one batched eks_smooth call.
    Returns {'left_df', 'right_df'} in the reference's layout."""
    return _paw_async(markers_list_left_cam, markers_list_right_cam, timestamps_left_cam,
                      timestamps_right_cam, keypoint_names, smooth_param, quantile_keep_pca,
                      opti=False)


def eks_opti_smoother_paw_asynchronous(
        markers_list_left_cam, markers_list_right_cam, timestamps_left_cam,
        timestamps_right_cam, keypoint_names, smooth_param, quantile_keep_pca):
    """The same model with the Newton forward filter instead of the RTS
    smoother (eks/multiview_pca_smoother.py:325-574)."""
    return _paw_async(markers_list_left_cam, markers_list_right_cam, timestamps_left_cam,
                      timestamps_right_cam, keypoint_names, smooth_param, quantile_keep_pca,
                      opti=True)


__all__ += ["ensemble_kalman_smoother_paw_asynchronous", "eks_opti_smoother_paw_asynchronous",
            "interp1d_linear"]
