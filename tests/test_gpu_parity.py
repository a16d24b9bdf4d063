"""GPU parity: the HIP path (through the C ABI) against the golden vectors
and the CPU oracle, on identical inputs.

Tolerances: the recursions are float64 in both paths but use different
(algebraically identical) update orders, so intermediates agree to ~1e-12
relative; outputs in pixel units are held to the north-star bound
max|d| < 1e-5 (BASELINE.json) and in practice agree to ~1e-10.
"""
import glob
import os
import warnings

import numpy as np
import pandas as pd
import pytest

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-5          # north-star tolerance on smoothed outputs (pixels)
INT_RTOL = 1e-8         # intermediates (mf, Vf, S, ms, Vs, CV)


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _close(a, b, rtol=INT_RTOL, atol=None):
    a = np.asarray(a)
    b = np.asarray(b)
    scale = max(1.0, float(np.nanmax(np.abs(b))) if b.size else 1.0)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=(atol if atol is not None else rtol * scale),
                               equal_nan=True)


# -------------------------------------------------------------------------
ENS = sorted(glob.glob(os.path.join(GOLDEN, "ensemble_*.npz")))


@pytest.mark.parametrize("path", ENS, ids=[os.path.basename(p)[:-4] for p in ENS])
def test_ensemble_golden(torch, path):
    from eks_amd import core
    g = np.load(path)
    mode = "median" if "median" in path else "mean"
    p, v = core.ensemble_array(g["stack"], mode)
    # selection and numpy-ordered sums: expected bit-exact
    np.testing.assert_array_equal(np.isnan(p), np.isnan(g["preds"]))
    np.testing.assert_allclose(p, g["preds"], rtol=0, atol=1e-12, equal_nan=True)
    np.testing.assert_allclose(v, g["vars"], rtol=1e-14, atol=1e-14, equal_nan=True)


def test_ensemble_dataframe_api(torch):
    from eks_amd import core
    g = np.load(os.path.join(GOLDEN, "ensemble_E5_median.npz"))
    keys = ["a", "b", "c"]
    dfs = [pd.DataFrame(g["stack"][e], columns=keys) for e in range(5)]
    preds, var, stacks, avg_d, var_d, stack_d = core.ensemble(dfs, keys)
    assert stacks.shape == g["stacks"].shape
    np.testing.assert_array_equal(stacks, g["stacks"])
    np.testing.assert_allclose(avg_d["b"], g["preds"][:, 1], atol=1e-12, equal_nan=True)
    np.testing.assert_array_equal(stack_d[3]["c"], g["stack"][3, :, 2])
    with pytest.raises(ValueError):
        core.ensemble(dfs, keys, mode="max")


@pytest.mark.parametrize("E", [1, 2, 3, 5, 7, 9, 16, 33])
def test_ensemble_member_counts_vs_oracle(torch, E):
    """Compiled (E <= 8) and runtime-E paths, float32 and float64 members."""
    from eks_amd import _lib, core
    from oracle import eks_oracle as O
    rng = np.random.default_rng(E)
    stack = rng.normal(200, 30, size=(E, 301, 4)).round(2)
    stack[:, 5, 0] = 7.25  # ties
    for mode in ("median", "mean"):
        p, v = core.ensemble_array(stack, mode)
        po, vo = O.ensemble_array(stack, mode)
        np.testing.assert_allclose(p, po, rtol=0, atol=1e-12)
        np.testing.assert_allclose(v, vo, rtol=1e-13, atol=1e-13)
    # float32 members through the raw C ABI, trajectory-minor layout
    B = 3
    s32 = rng.normal(200, 30, size=(301, E, 4, B)).astype(np.float32)  # (T, E, n, B)
    d = torch.from_numpy(s32).cuda()
    preds = torch.empty((B, 301, 4), dtype=torch.float64, device="cuda")
    var = torch.empty_like(preds)
    lib = _lib.load()
    _lib.check(lib.eks_ensemble(d.data_ptr(), _lib.EKS_F32, B, 301, E, 4, 1, E * 4 * B, 4 * B, B,
                                _lib.EKS_MEDIAN, preds.data_ptr(), var.data_ptr(),
                                _lib.stream_ptr()), "eks_ensemble")
    for b in range(B):
        po, vo = O.ensemble_array(np.transpose(s32[..., b], (1, 0, 2)).astype(np.float64))
        np.testing.assert_allclose(preds[b].cpu().numpy(), po, rtol=0, atol=1e-12)
        np.testing.assert_allclose(var[b].cpu().numpy(), vo, rtol=1e-13, atol=1e-13)


# -------------------------------------------------------------------------
CORE = sorted(glob.glob(os.path.join(GOLDEN, "core_*.npz")))


@pytest.mark.parametrize("path", CORE, ids=[os.path.basename(p)[:-4] for p in CORE])
def test_core_golden(torch, path):
    """filtering_pass / smooth_backward / kalman_dot drop-ins vs the reference."""
    from eks_amd import core
    g = np.load(path)
    R = g["R_in"].copy()
    mf, Vf, S = core.filtering_pass(g["y"], g["m0"], g["S0"], g["C"], R, g["A"], g["Q"], g["ev"])
    _close(mf, g["mf"])
    _close(Vf, g["Vf"])
    _close(S, g["S"])
    np.testing.assert_array_equal(R, g["R_out"])  # in-place mutation reproduced
    T = len(g["y"])
    if T >= 2:
        assert np.all(S[-1] == 0.0)
    ms, Vs, CV = core.smooth_backward(g["y"], mf, Vf, S, g["A"], g["Q"], g["C"])
    if T >= 2:
        _close(ms, g["ms"])
        _close(Vs, g["Vs"])
        _close(CV, g["CV"])
    assert CV.shape == (T - 1,) + g["A"].shape
    kd = core.kalman_dot(g["kd_vec_in"], g["S0"], g["C"], np.diag(g["ev"][0]))
    _close(kd, g["kd_vec"], rtol=1e-10)
    kd = core.kalman_dot(g["kd_mat_in"], g["S0"], g["C"], np.diag(g["ev"][0]))
    _close(kd, g["kd_mat"], rtol=1e-10)


def test_full_R_off_diagonal_vs_oracle(torch):
    """A non-diagonal caller R: off-diagonals are kept, diagonal replaced."""
    from eks_amd import core
    from oracle import eks_oracle as O
    g = np.load(os.path.join(GOLDEN, "core_rand_r3_n4_T257.npz"))
    R0 = np.eye(4) + 0.2 * (np.ones((4, 4)) - np.eye(4))
    R1, R2 = R0.copy(), R0.copy()
    a = core.filtering_pass(g["y"], g["m0"], g["S0"], g["C"], R1, g["A"], g["Q"], g["ev"])
    b = O.filtering_pass(g["y"], g["m0"], g["S0"], g["C"], R2, g["A"], g["Q"], g["ev"])
    for x, y in zip(a, b):
        _close(x, y)
    np.testing.assert_array_equal(R1, R2)


def test_nll_vs_oracle(torch):
    from eks_amd import core
    from oracle import eks_oracle as O
    for name in ("core_rand_r3_n8_T1000", "core_rand_r2_n2_T1000", "core_zero_var_r2_n2_T300"):
        g = np.load(os.path.join(GOLDEN, name + ".npz"))
        a = core.compute_nll(g["y"], g["m0"], g["S0"], g["C"], g["A"], g["Q"], g["ev"])
        b = O.compute_nll(g["y"], g["m0"], g["S0"], g["C"], g["A"], g["Q"], g["ev"])
        assert abs(a - b) <= 1e-9 * abs(b), (name, a, b)


def test_singular_raises_linalgerror(torch):
    from eks_amd import core
    y = np.zeros((4, 2))
    ev = np.zeros((4, 2))
    with pytest.raises(np.linalg.LinAlgError):
        core.filtering_pass(y, np.zeros(2), np.zeros((2, 2)), np.eye(2), np.eye(2), np.eye(2),
                            np.zeros((2, 2)), ev)
    with pytest.raises(np.linalg.LinAlgError):
        core.smooth_backward(y, np.zeros((4, 2)), np.zeros((4, 2, 2)), np.zeros((4, 2, 2)),
                             np.eye(2))


def test_nan_propagates_like_numpy(torch):
    from eks_amd import core
    from oracle import eks_oracle as O
    g = np.load(os.path.join(GOLDEN, "core_rand_r2_n2_T257.npz"))
    y = g["y"].copy()
    y[100, 1] = np.nan
    a = core.filtering_pass(y, g["m0"], g["S0"], g["C"], np.eye(2), g["A"], g["Q"], g["ev"])
    b = O.filtering_pass(y, g["m0"], g["S0"], g["C"], np.eye(2), g["A"], g["Q"], g["ev"])
    np.testing.assert_array_equal(np.isnan(a[0]), np.isnan(b[0]))
    _close(a[0][:100], b[0][:100])


# -------------------------------------------------------------------------
# fused hot path (eks_smooth)
# -------------------------------------------------------------------------
SV = sorted(glob.glob(os.path.join(GOLDEN, "singleview_*.npz")))


@pytest.mark.parametrize("path", SV, ids=[os.path.basename(p)[:-4] for p in SV])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_fused_singleview_golden(torch, path, dtype):
    """eks_smooth on the reference-generated single-view fixtures (model from
    the fixture), members as float64 and as float32 (they are f32 values)."""
    from eks_amd import batch
    g = np.load(path)
    obs = g["obs"]  # (E, T, 2)
    E, T, _ = obs.shape
    params = batch.pack_params(g["m0"], g["S0"], g["A"], g["Q"], g["C"], g["means"])
    npdt = np.float64 if dtype == "f64" else np.float32
    d = batch.make_time_major(obs[None], dtype=npdt)  # (1, T, E, 2) view
    res = batch.smooth(d, params, n=2, r=2, want_ms=True, want_nll=True)
    assert int(res["status"][0]) == 0
    out = res["out"][0].cpu().numpy()
    assert np.abs(out - g["out"]).max() < OUT_TOL
    _close(res["ms"][0].cpu().numpy(), g["ms"], rtol=1e-8)


@pytest.mark.parametrize("name", ["quant3", "quant5"])
def test_quantised_members_keep_reference_frames(torch, name):
    """Members on a 0.25 px grid (E = 3 and 5): the worst variances tie in
    large groups, so the percentile threshold equals many frames' values.
    The device ensemble (mean and variance scaled by 1/E and 1/E^2, within
    4 ulp of numpy's / E: ensemble.hpp) and the device fit (eks_fit, both
    selection paths) must keep exactly the frames the reference keeps
    (``good`` in the fixture, eks/multiview_pca_smoother.py:685-688's rule
    applied by tools/gen_golden.py with the reference's ensemble): the
    offsets are means over the kept frames, so one frame more or less moves
    them by ~1e-3 relative."""
    from eks_amd import _lib, batch
    g = np.load(os.path.join(GOLDEN, f"singleview_{name}.npz"))
    obs = g["obs"]  # (E, T, 2), float32-exact
    d = batch.make_time_major(obs[None], dtype=np.float32)
    import eks_amd.ops  # noqa: F401
    # the ensemble variances: within 4 ulp of the reference's (mean and
    # variance scaled by the rounded 1/E, 1/E^2 instead of numpy's divisions)
    _, ev = torch.ops.eks.ensemble(d, "median")
    np.testing.assert_allclose(ev[0].cpu().numpy(), g["ev"], rtol=9e-16, atol=0)
    for sel in (1, 2):
        prev = _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, sel)
        try:
            params, st = batch.fit(d, kind="singleview", n=2, r=2, smooth_param=float(g["s"]),
                                   quantile_keep=float(g["q"]))
        finally:
            _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, prev)
        p = params[0].cpu().numpy()
        off = p[-2:]
        np.testing.assert_allclose(off, g["means"], rtol=1e-12, atol=0)
        np.testing.assert_allclose(p[2:6].reshape(2, 2), g["S0"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(p[10:14].reshape(2, 2), g["Q"], rtol=1e-9, atol=1e-14)


def _oracle_smooth_batch(stacks, models, O):
    outs = []
    for st, m in zip(stacks, models):
        preds, ev = O.ensemble_array(st)
        y = preds - m["offset"]
        R = np.eye(len(m["offset"]))
        mf, Vf, S = O.filtering_pass(y, m["m0"], m["S0"], m["C"], R, m["A"], m["Q"], ev)
        ms, _, _ = O.smooth_backward(y, mf, Vf, S, m["A"])
        outs.append(ms @ m["C"].T + m["offset"])
    return outs


@pytest.mark.parametrize("algo", [1, 2, 3])
@pytest.mark.parametrize("r,n,E", [(2, 2, 5), (3, 4, 5), (3, 6, 4), (3, 8, 5), (2, 2, 11),
                                   (2, 2, 3)])
def test_fused_batch_vs_oracle(torch, r, n, E, algo):
    """B independent trajectories with different models and layouts, every
    algorithm (1 = sequential, 2 = time-parallel chunked scan, 3 = two-pass
    time-parallel; E = 11 is not compiled for algo 3, which then runs 2)."""
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    rng = np.random.default_rng(100 * r + n)
    B, T = 70, 400
    if n == 2:
        stacks = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3)  # (B, E, T, 2)
    else:
        stacks = synthetic.multiview_obs(rng, n // 2, E, T, K=B).transpose(2, 0, 1, 3)
    stacks = stacks.astype(np.float64)
    models = []
    for b in range(B):
        preds, ev = O.ensemble_array(stacks[b])
        if n == 2:
            p = O.singleview_params(preds, ev, 0.05, 25)
        else:
            p = O.multicam_params(preds, ev, 0.05, 25)
        p["offset"] = p["means"]
        models.append(p)
    params = batch.pack_params(np.stack([m["m0"] for m in models]),
                               np.stack([m["S0"] for m in models]),
                               np.stack([m["A"] for m in models]),
                               np.stack([m["Q"] for m in models]),
                               np.stack([m["C"] for m in models]),
                               np.stack([m["offset"] for m in models]))
    ref = _oracle_smooth_batch(list(stacks), models, O)
    flags = batch.model_flags(np.stack([m["A"] for m in models]),
                              np.stack([m["C"] for m in models]))
    # time-major float32 layout (the bench layout)
    d = batch.make_time_major(stacks, dtype=np.float32)
    res = batch.smooth(d, params, n=n, r=r, want_nll=True, algo=algo, flags=flags)
    out = res["out"].cpu().numpy()
    assert (res["status"] == 0).all()
    err = max(np.abs(out[b] - ref[b]).max() for b in range(B))
    assert err < OUT_TOL, err
    # trajectory-major float64 layout gives the same numbers
    d64 = torch.from_numpy(np.ascontiguousarray(stacks.transpose(0, 2, 1, 3))).cuda()  # (B,T,E,n)
    res2 = batch.smooth(d64, params, n=n, r=r, want_nll=True, algo=algo, flags=flags)
    np.testing.assert_allclose(res2["out"].cpu().numpy(), out, rtol=0, atol=1e-9)
    # without structure flags (general A, C code path) the same numbers
    res3 = batch.smooth(d, params, n=n, r=r, want_nll=True, algo=algo, flags=0)
    np.testing.assert_allclose(res3["out"].cpu().numpy(), out, rtol=0, atol=1e-9)
    # NLL per trajectory vs the oracle's definition
    for b in (0, B // 2, B - 1):
        preds, ev = O.ensemble_array(stacks[b])
        m = models[b]
        nll = O.compute_nll(preds - m["offset"], m["m0"], m["S0"], m["C"], m["A"], m["Q"], ev)
        assert abs(float(res["nll"][b]) - nll) <= 1e-9 * abs(nll)


@pytest.mark.parametrize("kind", ["singleview_heavy", "pupil_like", "multiview"])
def test_time_parallel_long_trajectories(torch, kind):
    """Few long trajectories (the configs 2/3/5 regime): the chunked scan
    (algo 2, hundreds of chunks per trajectory) against the sequential
    kernel on every trajectory and against the oracle on two of them."""
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    rng = np.random.default_rng(11)
    B, T, E = 6, 30000, 5
    if kind == "multiview":
        st = synthetic.multiview_obs(rng, 4, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float64)
        r, n = 3, 8
    elif kind == "pupil_like":
        st = np.stack([synthetic.pupil_obs(rng, E, T, a=0.999) for _ in range(B)]).astype(np.float64)
        r, n = 3, 8
    else:
        st = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float64)
        r, n = 2, 2
    models = []
    for b in range(B):
        preds, ev = O.ensemble_array(st[b])
        if kind == "singleview_heavy":
            p = O.singleview_params(preds, ev, 0.001, 25)
            p["offset"] = p["means"]
        elif kind == "multiview":
            p = O.multicam_params(preds, ev, 0.01, 25)
            p["offset"] = p["means"]
        else:
            p = O.pupil_params(preds, np.diag([0.9999, 0.999, 0.999]))
            p["offset"] = p["means"]
        models.append(p)
    stackp = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stackp("m0"), stackp("S0"), stackp("A"), stackp("Q"), stackp("C"),
                               stackp("offset"))
    flags = batch.model_flags(stackp("A"), stackp("C"))
    d = batch.make_time_major(st, dtype=np.float32)
    r1 = batch.smooth(d, params, n=n, r=r, algo=1, flags=flags, want_nll=True, check=True)
    o1 = r1["out"].cpu().numpy()
    n1 = r1["nll"].cpu().numpy()
    r2 = batch.smooth(d, params, n=n, r=r, algo=2, flags=flags, want_nll=True, check=True)
    o2 = r2["out"].cpu().numpy()
    n2 = r2["nll"].cpu().numpy()
    assert np.abs(o1 - o2).max() < 1e-8
    np.testing.assert_allclose(n2, n1, rtol=1e-10)
    r3 = batch.smooth(d, params, n=n, r=r, algo=3, flags=flags, want_nll=True)
    assert (r3["status"] == 0).all()
    assert np.abs(r3["out"].cpu().numpy() - o1).max() < 1e-8
    np.testing.assert_allclose(r3["nll"].cpu().numpy(), n1, rtol=1e-10)
    ref = _oracle_smooth_batch([st[0], st[B - 1]], [models[0], models[B - 1]], O)
    assert np.abs(o2[0] - ref[0]).max() < OUT_TOL
    assert np.abs(o2[B - 1] - ref[1]).max() < OUT_TOL


def test_model_flag_violation_is_reported(torch):
    from eks_amd import _lib, batch
    st = np.random.default_rng(3).normal(100, 3, size=(2, 5, 300, 2))
    A = np.array([[0.99, 0.0], [0.0, 1.0]])
    params = batch.pack_params(np.zeros(2), np.eye(2) * 10, A, np.eye(2) * 0.1, np.eye(2),
                               np.array([100.0, 100.0]))
    params = params.expand(2, -1).contiguous()
    res = batch.smooth(batch.make_time_major(st), params, n=2, r=2,
                       flags=_lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY)
    assert ((res["status"] & _lib.EKS_STATUS_BAD_MODEL) != 0).all()
    with pytest.raises(ValueError):
        batch.smooth(batch.make_time_major(st), params, n=2, r=2, check=True,
                     flags=_lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY)


def test_fused_edge_cases(torch):
    """T = 1, T = 2, zero-variance frames (all members agree) and NaN members."""
    from eks_amd import batch
    from oracle import eks_oracle as O
    rng = np.random.default_rng(7)
    for T in (1, 2, 3, 64, 65, 200):
        st = rng.normal(100, 5, size=(1, 4, T, 2))
        st[0, :, 0, 0] = 42.0   # exact agreement -> R_00 = 0 at t = 0
        m = dict(m0=np.zeros(2), S0=np.diag([30.0, 20.0]), A=np.eye(2),
                 Q=np.array([[0.5, 0.1], [0.1, 0.4]]), C=np.eye(2), offset=np.array([100., 100.]))
        params = batch.pack_params(m["m0"], m["S0"], m["A"], m["Q"], m["C"], m["offset"])
        ref = _oracle_smooth_batch([st[0]], [m], O)[0]
        for algo in (1, 2, 3):
            res = batch.smooth(batch.make_time_major(st), params, n=2, r=2, algo=algo, check=True)
            assert np.abs(res["out"][0].cpu().numpy() - ref).max() < OUT_TOL, (T, algo)
    st = rng.normal(100, 5, size=(1, 5, 50, 2))
    st[0, 2, 20, 1] = np.nan
    ref = _oracle_smooth_batch([st[0]], [m], O)[0]
    for algo in (1, 2, 3):
        res = batch.smooth(batch.make_time_major(st), params, n=2, r=2, algo=algo)
        out = res["out"][0].cpu().numpy()
        np.testing.assert_array_equal(np.isnan(out), np.isnan(ref))


# -------------------------------------------------------------------------
# entry points on the reference's own data (goldens committed by the reference)
# -------------------------------------------------------------------------
MC = sorted(glob.glob(os.path.join(GOLDEN, "multicam_*.npz")))


@pytest.mark.parametrize("path", MC, ids=[os.path.basename(p)[:-4] for p in MC])
def test_multicam_entry_point_golden(torch, path):
    from eks_amd.multiview_pca_smoother import ensemble_kalman_smoother_multi_cam
    g = np.load(path)
    stacks = g["stacks"]  # (V, E, T, 2)
    V, E = stacks.shape[:2]
    cams = [f"cam{c}" for c in range(V)]
    by_cam = [[pd.DataFrame(stacks[c, e], columns=["x", "y"]) for e in range(E)]
              for c in range(V)]
    dfs = ensemble_kalman_smoother_multi_cam(by_cam, "kp", float(g["s"]), float(g["q"]), cams)
    out = np.concatenate([dfs[f"{c}_df"].to_numpy()[:, :2] for c in cams], axis=1)
    assert np.abs(out - g["golden"]).max() < OUT_TOL
    assert np.abs(out - g["out"]).max() < OUT_TOL
    assert np.isnan(dfs["cam0_df"].to_numpy()[:, 2]).all()


def test_pupil_entry_point_golden(torch):
    from eks_amd.pupil_smoother import ensemble_kalman_smoother_pupil
    from eks_amd.fit import PUPIL_KEYS
    g = np.load(os.path.join(GOLDEN, "pupil_ibl.npz"))
    stack = g["stack"]
    dfs = [pd.DataFrame(stack[e], columns=list(PUPIL_KEYS)) for e in range(len(stack))]
    kps = [str(k) for k in g["keypoint_names"]]
    res = ensemble_kalman_smoother_pupil(dfs, kps, "ensemble-kalman_tracker", g["A"])
    mk = res["markers_df"].to_numpy()
    lat = res["latents_df"].to_numpy()
    assert np.nanmax(np.abs(mk - g["golden_markers"])) < OUT_TOL
    assert np.abs(lat - g["golden_latents"]).max() < OUT_TOL
    assert list(res["markers_df"].columns.get_level_values(1)[::3]) == kps


def test_singleview_entry_point(torch):
    from eks_amd.singleview_smoother import ensemble_kalman_smoother_single_view
    g = np.load(os.path.join(GOLDEN, "singleview_c1.npz"))
    obs = g["obs"]
    dfs = [pd.DataFrame(obs[e], columns=["nose_x", "nose_y"]) for e in range(len(obs))]
    res = ensemble_kalman_smoother_single_view(dfs, "nose", float(g["s"]), float(g["q"]))
    out = res["markers_df"].to_numpy()[:, :2]
    assert np.abs(out - g["out"]).max() < OUT_TOL
    assert np.isfinite(res["nll"])


@pytest.mark.parametrize("algo", [1, 2])
def test_filter_only_nll_matches_oracle(torch, algo):
    """Filter-only calls (out = NULL): candidate models of one trajectory
    sharing the member memory (batch stride 0) scored by their NLL."""
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    rng = np.random.default_rng(21)
    st = synthetic.pupil_obs(rng, 5, 3000).astype(np.float64)  # (E, T, 8)
    preds, ev = O.ensemble_array(st)
    grid = [(d, c) for d in (0.9, 0.99, 0.999) for c in (0.95, 0.999)]
    models = [O.pupil_params(preds, np.diag([d, c, c])) for d, c in grid]
    stackp = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stackp("m0"), stackp("S0"), stackp("A"), stackp("Q"), stackp("C"),
                               stackp("means"))
    obs = torch.from_numpy(st).cuda().permute(1, 0, 2).unsqueeze(0)
    scores = batch.nll(obs.expand(len(grid), -1, -1, -1), params, n=8, r=3, algo=algo)
    scores = scores.cpu().numpy()
    for i, m in enumerate(models):
        ref = O.compute_nll(preds - m["means"], m["m0"], m["S0"], m["C"], m["A"], m["Q"], ev)
        assert abs(scores[i] - ref) <= 1e-9 * abs(ref), (grid[i], scores[i], ref)


def test_pupil_smoothing_sweep(torch):
    from eks_amd.fit import PUPIL_KEYS
    from eks_amd.pupil_smoother import pupil_smoothing_sweep
    from eks_amd import synthetic
    st = synthetic.pupil_obs(np.random.default_rng(3), 5, 2000, a=0.99).astype(np.float64)
    dfs = [pd.DataFrame(st[e], columns=list(PUPIL_KEYS)) for e in range(5)]
    kps = ["pupil_top_r", "pupil_right_r", "pupil_bottom_r", "pupil_left_r"]
    res = pupil_smoothing_sweep(dfs, kps, "ensemble-kalman_tracker", [0.9, 0.99, 0.999],
                                [0.9, 0.99, 0.999])
    assert res["nll"].shape == (3, 3) and np.isfinite(res["nll"]).all()
    i, j = np.unravel_index(np.argmin(res["nll"]), res["nll"].shape)
    assert res["best"] == ([0.9, 0.99, 0.999][i], [0.9, 0.99, 0.999][j])
    assert res["markers_df"].shape == (2000, 12)


# -------------------------------------------------------------------------
# F3: Newton ("opti") filter, eks/newton_eks.py:115-148
NEWTON = sorted(glob.glob(os.path.join(GOLDEN, "newton_*.npz")))


@pytest.mark.parametrize("path", NEWTON, ids=[os.path.basename(p)[:-4] for p in NEWTON])
def test_newton_golden(torch, path):
    from eks_amd.newton_eks import kalman_newton_recursive
    g = np.load(path)
    it = int(g["max_iter"])
    res = kalman_newton_recursive(g["y"], g["mu0"], g["S0"], g["A"], g["B"], g["ev"], g["E"],
                                  max_iter=it)
    q = res if it == 1 else res[0]
    if it > 1:
        assert res[1].shape == (it,) and np.all(res[1] == 0)
    _close(q, g["q"])


@pytest.mark.parametrize("r,n,shared", [(1, 1, 0), (2, 2, 1), (3, 4, 0), (3, 8, 1), (4, 5, 0),
                                        (6, 8, 0), (5, 3, 1), (3, 10, 0), (3, 12, 1), (2, 64, 0)])
def test_newton_batch_vs_oracle(torch, r, n, shared):
    from eks_amd.newton_eks import newton_filter_batch
    from oracle import eks_oracle as O
    rng = np.random.default_rng(100 * r + n)
    Bn, T = 5, 150
    def spd(k, s):
        M = rng.normal(size=(k, k))
        return M @ M.T / k * s + np.eye(k) * 0.1 * s
    models = []
    for b in range(1 if shared else Bn):
        models.append(dict(mu0=rng.normal(size=r), S0=spd(r, 10.0),
                           A=np.eye(r) + 0.05 * rng.normal(size=(r, r)), E=spd(r, 0.5),
                           B=rng.normal(size=(n, r))))
    y = rng.normal(size=(Bn, T, n)) * 3
    ev = rng.uniform(0.05, 3.0, size=(Bn, T, n))
    st = (lambda k: models[0][k]) if shared else (lambda k: np.stack([m[k] for m in models]))
    q, status = newton_filter_batch(y, ev, st("mu0"), st("S0"), st("A"), st("B"), st("E"),
                                    max_iter=2)
    assert int(status.abs().sum().item()) == 0
    q = q.cpu().numpy()
    for b in range(Bn):
        m = models[0 if shared else b]
        ref, _ = O.kalman_newton_recursive(y[b], m["mu0"], m["S0"], m["A"], m["B"], ev[b], m["E"],
                                           max_iter=2)
        _close(q[b], ref)


def test_newton_singular_raises(torch):
    from eks_amd.newton_eks import kalman_newton_recursive
    g = np.load(NEWTON[-1])
    ev = g["ev"].copy()
    ev[5, 0] = 0.0
    with pytest.raises(np.linalg.LinAlgError):
        kalman_newton_recursive(g["y"], g["mu0"], g["S0"], g["A"], g["B"], ev, g["E"])
    with pytest.raises(np.linalg.LinAlgError):
        kalman_newton_recursive(g["y"], g["mu0"], 0 * g["S0"], g["A"], g["B"], g["ev"], g["E"])


def test_opti_multicam_golden(torch):
    from eks_amd.multiview_pca_smoother import eks_opti_smoother_multi_cam
    g = np.load(os.path.join(GOLDEN, "opti_mouse_paw2LF.npz"))
    stacks = g["stacks"]
    V, E = stacks.shape[:2]
    cams = ["top", "bot"]
    by_cam = [[pd.DataFrame(stacks[c, e], columns=["x", "y"]) for e in range(E)]
              for c in range(V)]
    dfs = eks_opti_smoother_multi_cam(by_cam, "paw2LF", float(g["s"]), float(g["q"]), cams)
    out = np.concatenate([dfs[f"{c}_df"].to_numpy()[:, :2] for c in cams], axis=1)
    assert np.abs(out - g["golden"]).max() < OUT_TOL
    assert np.isnan(dfs["top_df"].to_numpy()[:, 2]).all()


def test_opti_multicam_five_cameras_golden(torch):
    """eks_opti_smoother_multi_cam with 5 cameras (n = 10: the runtime-n
    Newton filter) against the reference run on the same synthetic members
    (tools/gen_golden.py bign)."""
    from eks_amd.multiview_pca_smoother import eks_opti_smoother_multi_cam
    g = np.load(os.path.join(GOLDEN, "opti_multicam_V5.npz"))
    st = g["stack"]                                    # (E, T, 2V)
    E, V = st.shape[0], st.shape[2] // 2
    cams = [f"cam{c}" for c in range(V)]
    by_cam = [[pd.DataFrame(st[e][:, 2 * c:2 * c + 2], columns=["paw_x", "paw_y"])
               for e in range(E)] for c in range(V)]
    dfs = eks_opti_smoother_multi_cam(by_cam, "paw", float(g["s"]), float(g["q"]), cams)
    out = np.concatenate([dfs[f"{c}_df"].to_numpy()[:, :2] for c in cams], axis=1)
    assert np.abs(out - g["out"]).max() < OUT_TOL


@pytest.mark.parametrize("n", [16, 64])
def test_forward_runtime_n_vs_oracle(torch, n):
    """The runtime-n dense forward and kalman_dot (n > 8: one wave per
    trajectory, the n x n solve in LDS) against the oracle at n = 16 and at
    the n = 64 maximum, with exact-agreement frames (ev = 0)."""
    from eks_amd import core
    from oracle import eks_oracle as O
    rng = np.random.default_rng(n)
    r, T = 3, 120
    A = np.eye(r) + 0.05 * rng.normal(size=(r, r))
    M = rng.normal(size=(r, r))
    Q = M @ M.T / r + 0.5 * np.eye(r)
    S0 = 20 * np.eye(r)
    C = rng.normal(size=(n, r)) * 2.0
    x = np.cumsum(rng.normal(size=(T, r)), axis=0)
    y = x @ C.T + rng.normal(size=(T, n))
    ev = rng.uniform(0.05, 4.0, size=(T, n))
    ev[rng.random(size=T) < 0.2, 0] = 0.0
    m0 = rng.normal(size=r)
    mf, Vf, S = core.filtering_pass(y, m0, S0, C, np.eye(n), A, Q, ev)
    mo, Vo, So = O.filtering_pass(y, m0, S0, C, np.eye(n), A, Q, ev)
    _close(mf, mo)
    _close(Vf, Vo)
    _close(S, So)
    ms, _, _ = core.smooth_backward(y, mf, Vf, S, A, Q, C)
    mso, _, _ = O.smooth_backward(y, mo, Vo, So, A)
    _close(ms, mso)
    v = rng.normal(size=(n, r))
    _close(core.kalman_dot(v, S0, C, np.diag(ev[1])), O.kalman_dot(v, S0, C, np.diag(ev[1])),
           rtol=1e-10)


def test_opti_pupil_golden(torch):
    from eks_amd.pupil_smoother import eks_opti_smoother_pupil
    from eks_amd.fit import PUPIL_KEYS
    g = np.load(os.path.join(GOLDEN, "opti_pupil_ibl.npz"))
    stack = g["stack"]
    dfs = [pd.DataFrame(stack[e], columns=list(PUPIL_KEYS)) for e in range(len(stack))]
    kps = ["pupil_top_r", "pupil_right_r", "pupil_bottom_r", "pupil_left_r"]
    res = eks_opti_smoother_pupil(dfs, kps, "ensemble-kalman_tracker", np.eye(3))
    assert np.abs(res["latents_df"].to_numpy() - g["golden_latents"]).max() < OUT_TOL


# -------------------------------------------------------------------------
# F2: batched model fit on the device (eks_fit) vs the host fit
def _unpack(p, n, r):
    o = 0
    out = {}
    for k, shp in (("m0", (r,)), ("S0", (r, r)), ("A", (r, r)), ("Q", (r, r)), ("C", (n, r)),
                   ("offset", (n,))):
        sz = int(np.prod(shp))
        out[k] = p[o:o + sz].reshape(shp)
        o += sz
    return out


@pytest.mark.parametrize("E,T,q,dtype", [(5, 3000, 25, "f32"), (3, 257, 10, "f64"),
                                         (4, 2000, 50, "f32"), (5, 1001, 100, "f64")])
def test_fit_singleview_vs_host(torch, E, T, q, dtype):
    from eks_amd import batch, fit, synthetic
    from eks_amd.core import ensemble_array
    rng = np.random.default_rng(E * T)
    B = 6
    st = np.stack([synthetic.singleview_obs(rng, E, T)[:, :, 0] for _ in range(B)])  # (B,E,T,2)
    st = st.astype(np.float32 if dtype == "f32" else np.float64)
    obs = torch.from_numpy(np.ascontiguousarray(st)).cuda().permute(0, 2, 1, 3)
    params, status = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=0.01,
                               quantile_keep=q)
    params = params.cpu().numpy()
    for b in range(B):
        preds, ev = ensemble_array(st[b].astype(np.float64))
        ref = fit.singleview_model(preds, ev, 0.01, q)
        got = _unpack(params[b], 2, 2)
        for k in ("m0", "S0", "A", "Q", "C", "offset"):
            _close(got[k], ref[k], rtol=1e-9)


def test_fit_singleview_one_kept_frame(torch):
    """q = 0 keeps exactly one frame (the minimum of the worst variance):
    offset = that frame's ensemble average, S0 = 0 (variance of one point)
    and Q = s * np.cov of zero consecutive-kept-frame differences, which
    numpy defines as NaN (ddof 1 with no pairs; the reference's np.cov at
    eks/multiview_pca_smoother.py:726-728 does the same).  The device fit
    must give exactly that, with status 0 (a kept frame exists)."""
    from eks_amd import batch, fit, synthetic
    from eks_amd.core import ensemble_array
    rng = np.random.default_rng(3500)
    E, T, B = 7, 500, 6
    st = np.stack([synthetic.singleview_obs(rng, E, T)[:, :, 0] for _ in range(B)]).astype(np.float64)
    obs = torch.from_numpy(np.ascontiguousarray(st)).cuda().permute(0, 2, 1, 3)
    params, status = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=0.01,
                               quantile_keep=0, check=False)
    assert (status.cpu().numpy() == 0).all()
    params = params.cpu().numpy()
    for b in range(B):
        preds, ev = ensemble_array(st[b])
        keep = np.argmin(ev.max(axis=1))
        got = _unpack(params[b], 2, 2)
        np.testing.assert_array_equal(got["offset"], preds[keep])
        np.testing.assert_array_equal(got["S0"], np.zeros((2, 2)))
        assert np.isnan(got["Q"]).all(), got["Q"]
        with np.errstate(all="ignore"), warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ref = fit.singleview_model(preds, ev, 0.01, 0)
        assert np.isnan(ref["Q"]).all()
        np.testing.assert_array_equal(ref["offset"], got["offset"])


@pytest.mark.parametrize("V,T", [(2, 2000), (4, 1500), (3, 700), (5, 3000), (6, 1500),
                                 (8, 700)])
def test_fit_multicam_vs_host(torch, V, T):
    """V >= 5 (n = 10..16) runs the wide kernels (k_fitw_*: 16-lane groups,
    one 256-thread block's Jacobi)."""
    from eks_amd import batch, fit, synthetic
    from eks_amd.core import ensemble_array
    rng = np.random.default_rng(V * T)
    K, E = 3, 5
    st = synthetic.multiview_obs(rng, V, E, T, K=K)  # (E, T, K, 2V) f32
    stacks = np.ascontiguousarray(st.transpose(2, 0, 1, 3))  # (K, E, T, 2V)
    obs = torch.from_numpy(stacks).cuda().permute(0, 2, 1, 3)
    n = 2 * V
    params, _ = batch.fit(obs, kind="multicam", n=n, r=3, smooth_param=0.01, quantile_keep=25)
    params = params.cpu().numpy()
    for k in range(K):
        preds, ev = ensemble_array(stacks[k].astype(np.float64))
        ref = fit.multicam_model(preds, ev, 0.01, 25)
        got = _unpack(params[k], n, 3)
        _close(got["offset"], ref["offset"], rtol=1e-9)
        _close(got["A"], ref["A"])
        # axes up to sign; S0 is sign-free, Q flips with the axis signs
        sgn = np.sign(np.sum(got["C"] * ref["C"], axis=0))
        _close(got["C"] * sgn, ref["C"], rtol=1e-7)
        _close(got["S0"], ref["S0"], rtol=1e-8)
        _close(got["Q"] * np.outer(sgn, sgn), ref["Q"], rtol=1e-7)


@pytest.mark.parametrize("V", [2, 6])
def test_fit_multicam_tiny_scale_pca(torch, V):
    """Members scaled by 2^-280 (scatter entries ~1e-165: d^2 + h^2 of a
    Jacobi rotation underflows, round-5 advisor finding): the PCA runs on
    exactly pre-scaled matrices (eks_fit.hip pca_scale), so the fit equals the
    unscaled one scaled by the same power of two -- axes, offsets, Q, S0.
    V = 2 runs k_fit_final, V = 6 the wide k_fitw_final."""
    from eks_amd import batch, synthetic
    rng = np.random.default_rng(40 + V)
    st = synthetic.multiview_obs(rng, V, 5, 600, K=2).astype(np.float64)  # (E, T, K, 2V)
    stacks = np.ascontiguousarray(st.transpose(2, 0, 1, 3))
    n = 2 * V
    sc = 2.0 ** -280
    fits = []
    for x in (stacks, stacks * sc):
        obs = torch.from_numpy(x).cuda().permute(0, 2, 1, 3)
        fits.append(batch.fit(obs, kind="multicam", n=n, r=3, smooth_param=0.01,
                              quantile_keep=25)[0].cpu().numpy())
    for k in range(2):
        a, b = _unpack(fits[0][k], n, 3), _unpack(fits[1][k], n, 3)
        assert np.isfinite(fits[1][k]).all()
        sgn = np.sign(np.sum(a["C"] * b["C"], axis=0))
        _close(b["C"] * sgn, a["C"], rtol=1e-12)
        _close(b["offset"] / sc, a["offset"], rtol=1e-12)
        _close(b["S0"] / sc ** 2, a["S0"], rtol=1e-12)
        _close(b["Q"] * np.outer(sgn, sgn) / sc ** 2, a["Q"], rtol=1e-12)


def test_fit_then_smooth_matches_singleview_golden(torch):
    """eks_fit + eks_smooth reproduce the committed single-view goldens."""
    from eks_amd import batch
    for path in sorted(glob.glob(os.path.join(GOLDEN, "singleview_*.npz"))):
        g = np.load(path)
        st = g["obs"]  # (E, T, 2)
        obs = torch.from_numpy(np.ascontiguousarray(st, dtype=np.float64)).cuda()
        obs = obs.permute(1, 0, 2).unsqueeze(0)
        params, _ = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=float(g["s"]),
                              quantile_keep=float(g["q"]))
        out = batch.smooth(obs, params, n=2, r=2, check=True)["out"][0].cpu().numpy()
        assert np.abs(out - g["out"]).max() < OUT_TOL, path


def test_fit_then_smooth_matches_multicam_golden(torch):
    from eks_amd import batch
    for path in sorted(glob.glob(os.path.join(GOLDEN, "multicam_*.npz"))):
        g = np.load(path)
        stacks = g["stacks"]  # (V, E, T, 2)
        st = np.concatenate(list(stacks), axis=2)  # (E, T, 2V)
        n = st.shape[2]
        obs = torch.from_numpy(np.ascontiguousarray(st, dtype=np.float64)).cuda()
        obs = obs.permute(1, 0, 2).unsqueeze(0)
        params, _ = batch.fit(obs, kind="multicam", n=n, r=3, smooth_param=float(g["s"]),
                              quantile_keep=float(g["q"]))
        out = batch.smooth(obs, params, n=n, r=3, check=True)["out"][0].cpu().numpy()
        assert np.abs(out - g["golden"]).max() < OUT_TOL, path


# -------------------------------------------------------------------------
# F4: asynchronous two-camera paw smoother
def test_interp1d_bit_exact(torch):
    from eks_amd.smoothers import interp1d_linear
    rng = np.random.default_rng(7)
    x = np.cumsum(rng.uniform(0.001, 0.05, size=500)) + 100.0
    y = rng.normal(size=(500, 6)) * 50
    y[17, 2] = np.nan
    xq = np.sort(rng.uniform(x[0], x[-1], size=300))
    xq[:3] = [x[0], x[10], x[-1]]  # exact sample times and both edges
    got = interp1d_linear(x, y, xq).cpu().numpy()
    ref = np.stack([np.interp(xq, x, y[:, c]) for c in range(6)], 1)
    assert np.array_equal(got, ref, equal_nan=True), np.nanmax(np.abs(got - ref))
    with pytest.raises(ValueError):
        interp1d_linear(x, y, np.array([x[0] - 1.0]))


@pytest.mark.parametrize("opti", [False, True])
def test_paw_async_golden(torch, opti):
    from eks_amd.multiview_pca_smoother import (ensemble_kalman_smoother_paw_asynchronous,
                                                eks_opti_smoother_paw_asynchronous)
    g = np.load(os.path.join(GOLDEN, "paw_async.npz"))
    cols = ['paw_l_x', 'paw_l_y', 'paw_l_likelihood', 'paw_r_x', 'paw_r_y', 'paw_r_likelihood']
    left = [pd.DataFrame(a, columns=cols) for a in g["left"]]
    right = [pd.DataFrame(a, columns=cols) for a in g["right"]]
    fn = eks_opti_smoother_paw_asynchronous if opti else ensemble_kalman_smoother_paw_asynchronous
    d = fn(left, right, g["tl"], g["tr"], ["paw_l", "paw_r"], float(g["s"]), float(g["q"]))
    k = "opti" if opti else "standard"
    for view in ("left", "right"):
        a = d[f"{view}_df"].to_numpy()
        b = g[f"{k}_{view}"]
        assert a.shape == b.shape
        assert np.nanmax(np.abs(a - b)) < OUT_TOL
        assert np.array_equal(np.isnan(a), np.isnan(b))


def test_torch_ops_match_batch_api(torch):
    import eks_amd.ops  # noqa: F401
    from eks_amd import batch, synthetic
    rng = np.random.default_rng(11)
    st = np.stack([synthetic.singleview_obs(rng, 5, 400)[:, :, 0] for _ in range(4)])
    obs = torch.from_numpy(np.ascontiguousarray(st)).cuda().permute(0, 2, 1, 3)
    params, _ = torch.ops.eks.fit(obs, "singleview", 2, 2, 0.01, 25.0, "median")
    out, status = torch.ops.eks.smooth(obs, params, 2, 2, "median", 0, 0)
    ref = batch.smooth(obs, params, n=2, r=2)["out"]
    assert int(status.abs().sum()) == 0
    assert torch.equal(out, ref.contiguous())
    p, v = torch.ops.eks.ensemble(obs, "median")
    assert p.shape == (4, 400, 2)
    nll = torch.ops.eks.nll(obs, params, 2, 2, "median", 0)
    assert torch.allclose(nll, batch.nll(obs, params, n=2, r=2), rtol=1e-12)
    # the operators are the C++ registrations of eks_amd/csrc/torch_ops.cpp
    # (TORCH_LIBRARY): no Python kernel anywhere in their dispatch
    for op in eks_amd.ops.OPS:
        dump = torch._C._dispatch_dump(f"eks::{op}")
        assert "CUDA: registered at" in dump and "torch_ops.cpp" in dump, dump
        assert ".py" not in dump, dump


def test_torch_ops_forward_backward_match_core(torch):
    """eks::forward / eks::backward (ensemble_kalman.filtering_pass /
    smooth_backward batched over trajectories) equal the drop-in core API on
    the reference-run golden systems."""
    import eks_amd.ops  # noqa: F401
    from eks_amd import core
    for path in CORE[:8]:
        g = np.load(path)
        y, ev = g["y"], g["ev"]
        mf_r, Vf_r, S_r = core.filtering_pass(y, g["m0"], g["S0"], g["C"], np.diag(np.diag(g["R_in"])),
                                              g["A"], g["Q"], ev)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()  # noqa: E731
        mf, Vf, S, nll, st = torch.ops.eks.forward(t(y)[None], t(ev)[None], t(g["m0"]), t(g["S0"]),
                                                   t(g["A"]), t(g["Q"]), t(g["C"]))
        assert int(st[0]) == 0, path
        np.testing.assert_array_equal(mf[0].cpu().numpy(), mf_r)
        np.testing.assert_array_equal(Vf[0].cpu().numpy(), Vf_r)
        np.testing.assert_array_equal(S[0].cpu().numpy(), S_r)
        ms_r, Vs_r, CV_r = core.smooth_backward(y, mf_r, Vf_r, S_r, g["A"])
        ms, Vs, CV, st2 = torch.ops.eks.backward(mf, Vf, S, t(g["A"]))
        assert int(st2[0]) == 0, path
        np.testing.assert_array_equal(ms[0].cpu().numpy(), ms_r)
        np.testing.assert_array_equal(Vs[0].cpu().numpy(), Vs_r)
        np.testing.assert_array_equal(CV[0].cpu().numpy(), CV_r)


def test_torch_ops_host_model_tensors_and_shapes(torch):
    """Model tensors on the host (numpy-derived) are moved to the call's device
    by eks::forward / backward / newton_filter -- same bits as device tensors
    (the Python shims they replace moved them too) -- and model arrays of the
    wrong shape are a RuntimeError before any kernel runs, never an
    out-of-bounds device read (round-4 advisor findings)."""
    import eks_amd.ops  # noqa: F401
    g = np.load(CORE[1])
    h = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))  # noqa: E731
    d = lambda a: h(a).cuda()  # noqa: E731
    y, ev = d(g["y"])[None], d(g["ev"])[None]
    ref = torch.ops.eks.forward(y, ev, d(g["m0"]), d(g["S0"]), d(g["A"]), d(g["Q"]), d(g["C"]))
    got = torch.ops.eks.forward(y, h(g["ev"])[None], h(g["m0"]), h(g["S0"]), h(g["A"]), h(g["Q"]),
                                h(g["C"]))
    for x0, x1 in zip(ref, got):
        assert torch.equal(x0, x1)
    mf, Vf, S = ref[:3]
    b0 = torch.ops.eks.backward(mf, Vf, S, d(g["A"]))
    b1 = torch.ops.eks.backward(mf, Vf.cpu(), S.cpu(), h(g["A"]))
    for x0, x1 in zip(b0, b1):
        assert torch.equal(x0, x1)
    r, n = g["m0"].shape[-1], g["y"].shape[-1]
    E = np.eye(r)
    q0 = torch.ops.eks.newton_filter(y, ev, d(g["m0"]), d(g["S0"]), d(g["A"]), d(g["C"]), d(E), 1)
    q1 = torch.ops.eks.newton_filter(y, ev, h(g["m0"]), h(g["S0"]), h(g["A"]), h(g["C"]), h(E), 1)
    assert torch.equal(q0[0], q1[0]) and torch.equal(q0[1], q1[1])
    bad = d(np.zeros((r + 1, r + 1)))
    with pytest.raises(RuntimeError, match="shape"):
        torch.ops.eks.forward(y, ev, d(g["m0"]), d(g["S0"]), bad, d(g["Q"]), d(g["C"]))
    with pytest.raises(RuntimeError, match="shape"):
        torch.ops.eks.forward(y, ev, d(g["m0"])[None].repeat(2, 1), d(g["S0"]), d(g["A"]),
                              d(g["Q"]), d(g["C"]))
    with pytest.raises(RuntimeError, match="shape"):
        torch.ops.eks.backward(mf, Vf[:, :-1], S, d(g["A"]))
    with pytest.raises(RuntimeError, match="shape"):
        torch.ops.eks.newton_filter(y, ev, d(g["m0"]), d(g["S0"]), d(g["A"]), d(np.zeros((n + 1, r))),
                                    d(E), 1)


# -------------------------------------------------------------------------
# fit -> smooth ensemble hand-off (EKS_YEV32 / EKS_YEV64): bit-identical
@pytest.mark.parametrize("kind,V,E,dtype,mode,algo", [
    ("singleview", 1, 5, "f32", "median", 0), ("singleview", 1, 5, "f32", "median", 1),
    ("singleview", 1, 5, "f32", "median", 3), ("singleview", 1, 4, "f64", "mean", 3),
    ("singleview", 1, 4, "f64", "median", 2), ("singleview", 1, 3, "f32", "mean", 0),
    ("multicam", 4, 5, "f32", "median", 0), ("multicam", 2, 3, "f64", "median", 1)])
def test_fit_yev_handoff_bit_exact(torch, kind, V, E, dtype, mode, algo):
    from eks_amd import batch, synthetic
    rng = np.random.default_rng(E * V + algo)
    K, T = 40, 3000
    if kind == "singleview":
        st = np.stack([synthetic.singleview_obs(rng, E, T)[:, :, 0] for _ in range(K)])
        n, r = 2, 2
    else:
        st = synthetic.multiview_obs(rng, V, E, T, K=K).transpose(2, 0, 1, 3)
        n, r = 2 * V, 3
    st = np.ascontiguousarray(st, dtype=np.float32 if dtype == "f32" else np.float64)
    obs = torch.from_numpy(st).cuda().permute(0, 2, 1, 3)   # (K, T, E, n)
    kw = dict(kind=kind, n=n, r=r, smooth_param=0.01, quantile_keep=25, mode=mode)
    p0, _ = batch.fit(obs, **kw)
    p1, _, yev = batch.fit(obs, keep_yev=True, **kw)
    assert torch.equal(p0, p1)
    a = batch.smooth(obs, p0, n=n, r=r, mode=mode, algo=algo, check=True)["out"]
    b = batch.smooth(yev, p1, n=n, r=r, mode=mode, algo=algo, check=True)["out"]
    assert torch.equal(a, b)
    y32 = dtype == "f32" and mode == "median" and E in (3, 5)
    assert yev.code == (2 if y32 else 3)


def test_algo3_batch_slices_bit_identical(torch):
    """algo 3's chained passes combine a unit's aggregate only with its
    neighbour's published value, so every operation's association order
    depends on T alone: smoothing a slice of the trajectories (ragged last
    64-trajectory group included) gives bit-identical results to smoothing
    all of them, and so does a second call (no timing dependence)."""
    from eks_amd import _lib, batch, synthetic
    rng = np.random.default_rng(21)
    B, T, E = 1100, 600, 5
    st = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float32)
    d = batch.make_time_major(st, dtype=np.float32)               # (B, T, E, 2) view
    params = batch.fit(d, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)[0]
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    full = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags, want_ms=True, want_nll=True)
    assert (full["status"] == 0).all()
    again = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags, want_ms=True, want_nll=True)
    assert torch.equal(again["out"], full["out"])
    assert torch.equal(again["nll"], full["nll"])
    for lo, hi in ((0, 70), (600, 700), (1030, 1100)):           # first half, boundary, second half
        part = batch.smooth(d[lo:hi], params[lo:hi].contiguous(), n=2, r=2, algo=3, flags=flags,
                            want_ms=True, want_nll=True)
        assert torch.equal(part["out"], full["out"][lo:hi]), (lo, hi)
        assert torch.equal(part["ms"], full["ms"][lo:hi]), (lo, hi)
        assert torch.equal(part["nll"], full["nll"][lo:hi]), (lo, hi)


@pytest.mark.parametrize("B", [1, 63, 300, 2100])
def test_algo3_chain_lengths(torch, B):
    """The chained passes over every chain length: T from one partial fine
    chunk (17 frames) to hundreds of coarse chunks, partial last fine and
    coarse chunks (T not a multiple of 16 / 64), one or many 64-trajectory
    groups with a ragged last one.  Against the sequential recursion (algo 1):
    outputs and smoothed means < 1e-8, NLL rtol 1e-10, no status bits."""
    from eks_amd import _lib, batch, synthetic
    rng = np.random.default_rng(40 + B)
    E = 5
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    for T in (17, 64, 65, 700, 4003):
        if B * T > 2100 * 700:
            continue
        st = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float32)
        d = batch.make_time_major(st, dtype=np.float32)
        params = batch.fit(d, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)[0]
        ref = batch.smooth(d, params, n=2, r=2, algo=1, flags=flags, want_ms=True, want_nll=True)
        got = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags, want_ms=True, want_nll=True)
        assert _lib.load().eks_smooth_algo(B, T, 2, 2, E, 3) == 3, T
        assert (got["status"] == 0).all(), T
        assert float((got["out"] - ref["out"]).abs().max()) < 1e-8, T
        assert float((got["ms"] - ref["ms"]).abs().max()) < 1e-8, T
        torch.testing.assert_close(got["nll"], ref["nll"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("kind,B,T", [("singleview", 1, 100), ("singleview", 5, 3000),
                                      ("singleview", 300, 5000), ("singleview", 17, 30000),
                                      ("multicam", 3, 20000), ("multicam", 40, 2000)])
def test_filter_only_closed_form_nll(torch, kind, B, T):
    """Filter-only calls take each chunk's NLL share in closed form from its
    filtering element and the chunk's start state (kf_steps.hpp
    elem_nll_share) instead of re-running the filter: it must equal the
    sequential filter's NLL (algo 1) to rtol 1e-10, for short (sequential
    K2) and long (wave-parallel K2) chunk chains, own and shared members."""
    from eks_amd import _lib, batch, synthetic
    rng = np.random.default_rng(B * 7 + T)
    if kind == "singleview":
        st = synthetic.singleview_obs(rng, 5, T, K=B).transpose(2, 0, 1, 3)   # (B, E, T, 2)
        n, r, flags = 2, 2, _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    else:
        st = synthetic.multiview_obs(rng, 3, 5, T, K=B).transpose(2, 0, 1, 3)  # (B, E, T, 6)
        n, r, flags = 6, 3, _lib.EKS_MODEL_A_IDENTITY
    obs = batch.make_time_major(st, dtype=np.float32)
    params, _ = batch.fit(obs, kind=kind, n=n, r=r, smooth_param=0.01, quantile_keep=25)
    ref = batch.smooth(obs, params, n=n, r=r, algo=1, flags=flags, want_nll=True)["nll"]
    got = batch.nll(obs, params, n=n, r=r, algo=2, flags=flags)
    rel = float(((got - ref) / ref.abs()).abs().max())
    assert rel < 1e-10, rel
    # one recording scored under B candidate models (members shared, stride 0)
    one = obs[:1].expand(B, -1, -1, -1)
    p1 = params[:1].expand(B, -1).contiguous()
    p1[:, -n:] += torch.arange(B, dtype=torch.float64, device=p1.device)[:, None] * 0.25
    ref1 = batch.smooth(one, p1, n=n, r=r, algo=1, flags=flags, want_nll=True)["nll"]
    got1 = batch.nll(one, p1, n=n, r=r, algo=2, flags=flags)
    rel1 = float(((got1 - ref1) / ref1.abs()).abs().max())
    assert rel1 < 1e-10, rel1
    # and smoothed under them (k_c0_shared: the shared ensemble computed once)
    o2 = batch.smooth(one, p1, n=n, r=r, algo=2, flags=flags)["out"]
    o1 = batch.smooth(one, p1, n=n, r=r, algo=1, flags=flags)["out"]
    assert float((o2 - o1).abs().max()) < 1e-8


def test_algo2_chained_scans_deterministic(torch):
    """Few long trajectories run algo 2's chained chunk scans with many
    blocks per trajectory (k_c2_fscan_g / k_c4_bscan_g: block hand-offs whose
    timing varies run to run): the association order is fixed by (NC, G), so
    repeated calls give the same bits, smoothed means, NLL and the
    filter-only NLL alike, and they match the sequential kernel."""
    from eks_amd import _lib, batch, synthetic
    rng = np.random.default_rng(5)
    B, T = 3, 120000
    st = synthetic.singleview_obs(rng, 5, T, K=B).transpose(2, 0, 1, 3)
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    obs = batch.make_time_major(st, dtype=np.float32)
    params, _ = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)
    runs = [batch.smooth(obs, params, n=2, r=2, algo=2, flags=flags, want_nll=True, check=True)
            for _ in range(3)]
    for r_ in runs[1:]:
        assert torch.equal(r_["out"], runs[0]["out"])
        assert torch.equal(r_["nll"], runs[0]["nll"])
    nl = [batch.nll(obs, params, n=2, r=2, algo=2, flags=flags) for _ in range(3)]
    assert torch.equal(nl[1], nl[0]) and torch.equal(nl[2], nl[0])
    ref = batch.smooth(obs, params, n=2, r=2, algo=1, flags=flags, want_nll=True)
    assert float((runs[0]["out"] - ref["out"]).abs().max()) < 1e-8
    torch.testing.assert_close(runs[0]["nll"], ref["nll"], rtol=1e-10, atol=0)
    torch.testing.assert_close(nl[0], ref["nll"], rtol=1e-10, atol=0)
