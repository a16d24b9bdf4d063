"""EKS_MODEL_PUPIL kernels (sparse pupil C, diagonal A / Q, the two pairs of
equal measurement rows folded into one observation each) against the dense
r = 3, n = 8 kernels and the oracle (eks/pupil_smoother.py:130-191).

The folded updates are the same Bayesian update in another order, so the
outputs agree with the dense path to rounding: < 1e-8 px, NLL rtol 1e-10.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PX = 1e-8
NLL_RTOL = 1e-10


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _models(preds_list, a_list):
    from oracle import eks_oracle as O
    ms = []
    for preds, a in zip(preds_list, a_list):
        p = O.pupil_params(preds, np.diag(a))
        p["offset"] = p["means"]
        ms.append(p)
    return ms


def _pack(models):
    from eks_amd import batch
    stk = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stk("m0"), stk("S0"), stk("A"), stk("Q"), stk("C"), stk("offset"))
    return params, batch.model_flags(stk("A"), stk("C"), stk("Q"))


@pytest.mark.parametrize("algo", [1, 2, 3])
def test_pupil_kernels_match_dense(torch, algo):
    from eks_amd import _lib, batch, synthetic
    from oracle import eks_oracle as O
    rng = np.random.default_rng(algo)
    B, E, T = 4, 5, 20000
    st = np.stack([synthetic.pupil_obs(rng, E, T, a=0.99) for _ in range(B)])
    st = st.astype(np.float32).astype(np.float64)   # what the device reads (f32 members)
    st[1, 2, 500:503] = np.nan                      # a NaN member: NaN frames as numpy
    st[2, :, 700, 0] = st[2, 0, 700, 0]             # exact agreement in one of a folded pair
    st[3, :, 900, 5] = st[3, 0, 900, 5]
    preds = [O.ensemble_array(st[b])[0] for b in range(B)]
    models = _models(preds, [[0.999, 0.99, 0.99], [0.99, 0.999, 0.999],
                             [0.9999, 0.95, 0.95], [0.9, 0.9, 0.9]])
    params, flags = _pack(models)
    assert flags == _lib.EKS_MODEL_PUPIL
    d = batch.make_time_major(st, dtype=np.float32)
    dense = batch.smooth(d, params, n=8, r=3, algo=algo, flags=0, want_nll=algo != 3,
                         want_ms=True, check=False)
    sparse = batch.smooth(d, params, n=8, r=3, algo=algo, flags=flags, want_nll=algo != 3,
                          want_ms=True, check=False)
    np.testing.assert_array_equal(sparse["status"].cpu().numpy(), dense["status"].cpu().numpy())
    o_d, o_s = dense["out"].cpu().numpy(), sparse["out"].cpu().numpy()
    np.testing.assert_array_equal(np.isnan(o_s), np.isnan(o_d))
    assert np.nanmax(np.abs(o_s - o_d)) < PX
    assert np.nanmax(np.abs(sparse["ms"].cpu().numpy() - dense["ms"].cpu().numpy())) < PX
    if algo != 3:
        n_d, n_s = dense["nll"].cpu().numpy(), sparse["nll"].cpu().numpy()
        fin = np.isfinite(n_d)
        np.testing.assert_array_equal(np.isfinite(n_s), fin)
        np.testing.assert_allclose(n_s[fin], n_d[fin], rtol=NLL_RTOL)
    # and the oracle (the reference's dense per-step solve) on a clean trajectory
    ref = O.pupil_smooth(st[0], models[0]["A"])
    got = batch.smooth(d[:1], params[:1].contiguous(), n=8, r=3, algo=algo, flags=flags,
                       check=True)["out"][0].cpu().numpy()
    assert np.abs(got - ref[0]).max() < 1e-5


def test_pupil_sweep_nll_matches_dense(torch):
    """The config-5 call: candidate models of one recording (members shared,
    batch stride 0), filter only (closed-form NLL shares)."""
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    st = synthetic.pupil_obs(np.random.default_rng(9), 5, 60000, a=0.99).astype(np.float64)
    preds, ev = O.ensemble_array(st)
    grid = [(dd, c) for dd in (0.9, 0.99, 0.999, 0.9999) for c in (0.9, 0.99, 0.999, 0.9999)]
    models = _models([preds] * len(grid), [[dd, c, c] for dd, c in grid])
    params, flags = _pack(models)
    obs = torch.from_numpy(st.astype(np.float32)).cuda().permute(1, 0, 2).unsqueeze(0)
    cobs = obs.expand(len(grid), -1, -1, -1)
    for algo in (1, 2):
        dense = batch.nll(cobs, params, n=8, r=3, algo=algo, flags=0).cpu().numpy()
        sparse = batch.nll(cobs, params, n=8, r=3, algo=algo, flags=flags).cpu().numpy()
        np.testing.assert_allclose(sparse, dense, rtol=NLL_RTOL)
    pre, evp = O.ensemble_array(st[:, :5000].astype(np.float32).astype(np.float64))
    for i in (0, 7, 15):
        m = models[i]
        want = O.compute_nll(pre - m["offset"], m["m0"], m["S0"], m["C"], m["A"], m["Q"], evp)
        got = float(batch.nll(obs[:, :5000], params[i:i + 1].contiguous(), n=8, r=3,
                              flags=flags)[0])
        assert abs(got - want) <= 1e-9 * abs(want), (i, got, want)


def test_pupil_sweep_64_candidates_scalar_planes(torch):
    """64 candidates (a multiple of 64: every wave of the sweep's K1 reads one
    step of the shared y / ev planes, through scalar loads) against the same
    members handed over per candidate (no sharing: the vector path) and the
    oracle; the 16-candidate sweep above covers the per-lane loads."""
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    T = 20000
    st = synthetic.pupil_obs(np.random.default_rng(11), 5, T, a=0.99).astype(np.float64)
    preds, ev = O.ensemble_array(st)
    dg = 1.0 - np.geomspace(1e-4, 1e-1, 8)
    grid = [(dd, c) for dd in dg for c in dg]
    models = _models([preds] * len(grid), [[dd, c, c] for dd, c in grid])
    params, flags = _pack(models)
    obs = torch.from_numpy(st.astype(np.float32)).cuda().permute(1, 0, 2).unsqueeze(0)
    shared = obs.expand(len(grid), -1, -1, -1)      # batch stride 0
    copies = shared.contiguous()                    # one copy per candidate
    for algo in (0, 2):
        a = batch.nll(shared, params, n=8, r=3, algo=algo, flags=flags).cpu().numpy()
        b = batch.nll(copies, params, n=8, r=3, algo=algo, flags=flags).cpu().numpy()
        np.testing.assert_allclose(a, b, rtol=1e-12)
    pre, evp = O.ensemble_array(st.astype(np.float32).astype(np.float64))
    for i in (0, 27, 63):
        m = models[i]
        want = O.compute_nll(pre - m["offset"], m["m0"], m["S0"], m["C"], m["A"], m["Q"], evp)
        assert abs(float(a[i]) - want) <= 1e-9 * abs(want), (i, float(a[i]), want)


def test_pupil_both_rows_exact_is_singular(torch):
    """Both members of a folded pair observed exactly (zero ensemble variance
    in columns 5 and 7 at one frame): the reference's S has two equal rows
    and zero noise there -- singular; the pupil kernels flag it."""
    from eks_amd import _lib, batch, synthetic
    from oracle import eks_oracle as O
    st = synthetic.pupil_obs(np.random.default_rng(4), 5, 3000, a=0.99).astype(np.float64)
    st[:, 1000, 5] = st[0, 1000, 5]
    st[:, 1000, 7] = st[0, 1000, 7]
    params, flags = _pack(_models([O.ensemble_array(st)[0]], [[0.99, 0.99, 0.99]]))
    d = batch.make_time_major(st[None], dtype=np.float32)
    for algo in (1, 2):
        res = batch.smooth(d, params, n=8, r=3, algo=algo, flags=flags, check=False)
        assert int(res["status"][0]) & (_lib.EKS_STATUS_SINGULAR | _lib.EKS_STATUS_SCAN), algo


def test_pupil_flag_violation_is_reported(torch):
    from eks_amd import _lib, batch, synthetic
    from oracle import eks_oracle as O
    st = synthetic.pupil_obs(np.random.default_rng(5), 5, 2000, a=0.99).astype(np.float64)
    m = _models([O.ensemble_array(st)[0]], [[0.99, 0.99, 0.99]])[0]
    d = batch.make_time_major(st[None], dtype=np.float32)
    for bad in ("A", "C", "Q"):
        mm = dict(m)
        mm[bad] = m[bad].copy()
        mm[bad][0, 1] += 0.01
        p = batch.pack_params(mm["m0"], mm["S0"], mm["A"], mm["Q"], mm["C"], mm["offset"])
        res = batch.smooth(d, p, n=8, r=3, algo=2, flags=_lib.EKS_MODEL_PUPIL, check=False)
        assert int(res["status"][0]) & _lib.EKS_STATUS_BAD_MODEL, bad
