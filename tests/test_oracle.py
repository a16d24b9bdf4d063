"""Pin the CPU oracle to the reference's golden vectors (CPU only).

The fixtures in tests/golden/ were produced by running the reference itself
(tools/gen_golden.py); the multicam/pupil fixtures also carry the reference's
own committed outputs (data/mirror-mouse/output/eks.csv,
data/misc/pupil-test/kalman_smoothed_*.csv, mirror-fish eks/ outputs).
"""
import glob
import os

import numpy as np
import pytest

from oracle import eks_oracle as O
from tests.conftest import GOLDEN

CORE = sorted(glob.glob(os.path.join(GOLDEN, "core_*.npz")))


@pytest.mark.parametrize("path", CORE, ids=[os.path.basename(p)[:-4] for p in CORE])
def test_core_filter_smoother(path):
    g = np.load(path)
    R = g["R_in"].copy()
    mf, Vf, S = O.filtering_pass(g["y"], g["m0"], g["S0"], g["C"], R, g["A"], g["Q"], g["ev"])
    np.testing.assert_allclose(mf, g["mf"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(Vf, g["Vf"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(S, g["S"], rtol=0, atol=1e-9)
    assert np.all(S[-1] == 0) or len(S) == 1  # quirk: S[T-1] never written
    np.testing.assert_array_equal(R, g["R_out"])  # quirk: R mutated in place
    T = g["y"].shape[0]
    if T >= 2:
        ms, Vs, CV = O.smooth_backward(g["y"], mf, Vf, S, g["A"], g["Q"], g["C"])
        np.testing.assert_allclose(ms, g["ms"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(Vs, g["Vs"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(CV, g["CV"], rtol=0, atol=1e-9)
    kd = O.kalman_dot(g["kd_vec_in"], g["S0"], g["C"], np.diag(g["ev"][0]))
    np.testing.assert_allclose(kd, g["kd_vec"], rtol=1e-12, atol=1e-12)
    kd = O.kalman_dot(g["kd_mat_in"], g["S0"], g["C"], np.diag(g["ev"][0]))
    np.testing.assert_allclose(kd, g["kd_mat"], rtol=1e-12, atol=1e-12)


ENS = sorted(glob.glob(os.path.join(GOLDEN, "ensemble_*.npz")))


@pytest.mark.parametrize("path", ENS, ids=[os.path.basename(p)[:-4] for p in ENS])
def test_ensemble(path):
    g = np.load(path)
    mode = "median" if "median" in path else "mean"
    p, v = O.ensemble_array(g["stack"], mode)
    np.testing.assert_allclose(p, g["preds"], rtol=0, atol=1e-12, equal_nan=True)
    np.testing.assert_allclose(v, g["vars"], rtol=0, atol=1e-12, equal_nan=True)


def test_ensemble_bad_mode():
    with pytest.raises(ValueError):
        O.ensemble_array(np.zeros((3, 4, 2)), "mode-that-does-not-exist")


SV = sorted(glob.glob(os.path.join(GOLDEN, "singleview_*.npz")))


@pytest.mark.parametrize("path", SV, ids=[os.path.basename(p)[:-4] for p in SV])
def test_singleview(path):
    g = np.load(path)
    out, p, _ = O.singleview_smooth(g["obs"], float(g["s"]), float(g["q"]))
    np.testing.assert_allclose(p["Q"], g["Q"], rtol=1e-12)
    np.testing.assert_allclose(p["S0"], g["S0"], rtol=1e-12)
    np.testing.assert_allclose(out, g["out"], rtol=0, atol=1e-9)


MC = sorted(glob.glob(os.path.join(GOLDEN, "multicam_*.npz")))


@pytest.mark.parametrize("path", MC, ids=[os.path.basename(p)[:-4] for p in MC])
def test_multicam(path):
    g = np.load(path)
    stacks = list(g["stacks"])  # per camera (E, T, 2)
    out, _, _ = O.multicam_smooth(stacks, float(g["s"]), float(g["q"]))
    np.testing.assert_allclose(out, g["out"], rtol=0, atol=1e-8)      # reference re-run
    np.testing.assert_allclose(out, g["golden"], rtol=0, atol=1e-8)   # committed golden


def test_pupil():
    g = np.load(os.path.join(GOLDEN, "pupil_ibl.npz"))
    markers, latents, _, _ = O.pupil_smooth(g["stack"], g["A"])
    # reference output column order: top, right, bottom, left with NaN likelihood
    order = [0, 1, 4, 5, 2, 3, 6, 7]
    mk = g["markers"].reshape(len(markers), 4, 3)[:, :, :2].reshape(len(markers), 8)
    np.testing.assert_allclose(markers[:, order], mk, rtol=0, atol=1e-9)
    np.testing.assert_allclose(latents, g["latents"], rtol=0, atol=1e-9)
    gm = g["golden_markers"].reshape(len(markers), 4, 3)[:, :, :2].reshape(len(markers), 8)
    np.testing.assert_allclose(markers[:, order], gm, rtol=0, atol=1e-9)
    np.testing.assert_allclose(latents, g["golden_latents"], rtol=0, atol=1e-9)


def test_nll_matches_dense_definition():
    """The NLL restatement agrees with a direct dense multivariate-normal
    evaluation of the innovation sequence (self-consistency; parity unpinned)."""
    g = np.load(os.path.join(GOLDEN, "core_rand_r3_n4_T257.npz"))
    nll = O.compute_nll(g["y"], g["m0"], g["S0"], g["C"], g["A"], g["Q"], g["ev"])
    from scipy.stats import multivariate_normal
    mf, S = g["mf"], g["S"]
    tot = 0.0
    for t in range(len(mf)):
        pm = g["m0"] if t == 0 else g["A"] @ mf[t - 1]
        pP = g["S0"] if t == 0 else S[t - 1]
        sig = np.diag(g["ev"][t]) + g["C"] @ pP @ g["C"].T
        tot -= multivariate_normal(g["C"] @ pm, sig).logpdf(g["y"][t])
    assert abs(nll - tot) < 1e-8 * abs(tot)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "newton_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_newton(path):
    g = np.load(path)
    it = int(g["max_iter"])
    res = O.kalman_newton_recursive(g["y"], g["mu0"], g["S0"], g["A"], g["B"], g["ev"], g["E"],
                                    max_iter=it)
    q = res if it == 1 else res[0]
    if it > 1:
        assert np.all(res[1] == 0.0)  # the reference's in-place alias makes the loss 0
    np.testing.assert_allclose(q, g["q"], rtol=0, atol=1e-9 * max(1.0, np.abs(g["q"]).max()))


def test_newton_multicam_opti():
    g = np.load(os.path.join(GOLDEN, "opti_mouse_paw2LF.npz"))
    out, _, _ = O.multicam_opti_smooth(list(g["stacks"]), float(g["s"]), float(g["q"]))
    np.testing.assert_allclose(out, g["out"], rtol=0, atol=1e-8)
    np.testing.assert_allclose(out, g["golden"], rtol=0, atol=1e-8)


def test_newton_pupil_opti():
    g = np.load(os.path.join(GOLDEN, "opti_pupil_ibl.npz"))
    _, latents, _, _ = O.pupil_opti_smooth(g["stack"])
    np.testing.assert_allclose(latents, g["latents"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(latents, g["golden_latents"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("opti", [False, True])
def test_paw_async(opti):
    g = np.load(os.path.join(GOLDEN, "paw_async.npz"))
    left, right = O.paw_async_smooth(g["left"], g["right"], g["tl"], g["tr"], float(g["s"]),
                                     float(g["q"]), opti=opti)
    k = "opti" if opti else "standard"
    exp_l = g[f"{k}_left"].reshape(len(left), 2, 3)[:, :, :2].reshape(len(left), 4)
    exp_r = g[f"{k}_right"].reshape(len(right), 2, 3)[:, :, :2].reshape(len(right), 4)
    np.testing.assert_allclose(left, exp_l, rtol=0, atol=1e-8)
    np.testing.assert_allclose(right, exp_r, rtol=0, atol=1e-8)
    assert np.isnan(g[f"{k}_left"][:, 2]).all()


def test_paw_select_and_interp():
    g = np.load(os.path.join(GOLDEN, "paw_async.npz"))
    from scipy.interpolate import interp1d
    sel = O.paw_async_select(g["tl"], g["tr"])
    assert len(sel) > 250
    y = g["right"][0][:, 0]
    a = interp1d(g["tr"], y)(g["tl"][sel])
    assert np.array_equal(a, np.interp(g["tl"][sel], g["tr"], y))
