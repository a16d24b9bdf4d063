"""eks_smooth's runtime-n kernel (algo 4, eks_shape_rt.hip): any number of
observed coordinates -- the multi-camera model with V > 4 cameras, which the
reference accepts (eks/multiview_pca_smoother.py:641-666) -- against the
oracle, and equal to the compiled general-C kernels (to ~1 ulp) where both exist.
"""
import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("V,T", [(5, 600), (8, 300)])
def test_multicam_wrapper_many_cameras_vs_oracle(torch, V, T):
    from eks_amd import synthetic
    from eks_amd.multiview_pca_smoother import ensemble_kalman_smoother_multi_cam
    from oracle import eks_oracle as O
    E = 5
    st = synthetic.multiview_obs(np.random.default_rng(V), V, E, T, K=1)[:, :, 0, :]  # (E,T,2V)
    st = st.astype(np.float64)
    cams = [f"cam{c}" for c in range(V)]
    markers = [[pd.DataFrame(st[e][:, 2 * c:2 * c + 2], columns=["x", "y"]) for e in range(E)]
               for c in range(V)]
    res = ensemble_kalman_smoother_multi_cam(markers, "paw", 0.01, 25, cams)
    got = np.concatenate([res[c + "_df"].to_numpy()[:, :2] for c in cams], axis=1)
    ref, _, _ = O.multicam_smooth([st[:, :, 2 * c:2 * c + 2] for c in range(V)], 0.01, 25)
    assert np.abs(got - ref).max() < 1e-5


@pytest.fixture
def rt_form():
    """eks_debug_set(EKS_DBG_RT_FORM, v) for one test, reset afterwards."""
    from eks_amd import _lib
    yield lambda v: _lib.debug_set(_lib.EKS_DBG_RT_FORM, v)
    _lib.debug_set(_lib.EKS_DBG_RT_FORM, 0)


@pytest.mark.parametrize("r,n,E", [(2, 2, 5), (2, 2, 7), (3, 8, 5), (3, 6, 4), (3, 12, 5),
                                   (3, 16, 3)])
def test_runtime_n_kernel_equals_compiled(torch, rt_form, r, n, E):
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    rt_form(1)  # the one-lane-per-trajectory form: the compiled kernels' update order
    rng = np.random.default_rng(r * 100 + n * 10 + E)
    B, T = 70, 500
    if r == 2:
        st = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3)
    else:
        st = synthetic.multiview_obs(rng, n // 2, E, T, K=B).transpose(2, 0, 1, 3)
    models = []
    for b in range(B):
        preds, ev = O.ensemble_array(st[b].astype(np.float64))
        p = O.singleview_params(preds, ev, 0.01, 25) if r == 2 else \
            O.multicam_params(preds, ev, 0.01, 25)
        models.append(p)
    stk = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stk("m0"), stk("S0"), stk("A"), stk("Q"), stk("C"), stk("means"))
    d = batch.make_time_major(st, dtype=np.float32)
    r1 = batch.smooth(d, params, n=n, r=r, algo=1, flags=0, want_nll=True, want_ms=True,
                      check=True)
    r4 = batch.smooth(d, params, n=n, r=r, algo=4, flags=0, want_nll=True, want_ms=True,
                      check=True)
    # same update order as the compiled general-C kernel; the ensemble comes
    # from the runtime-E reduction and the compiler contracts differently, so
    # the two agree to ~1 ulp rather than bit for bit
    for k in ("out", "ms", "nll"):
        np.testing.assert_allclose(r4[k].cpu().numpy(), r1[k].cpu().numpy(), rtol=1e-12,
                                   atol=1e-10, err_msg=k)


def test_runtime_n_nll_and_filter_only(torch):
    """n = 10 (five cameras): smoothed output, NLL and the filter-only call
    against the oracle's filtering_pass / compute_nll."""
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    rng = np.random.default_rng(31)
    B, E, T, n = 3, 5, 800, 10
    st = synthetic.multiview_obs(rng, 5, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float64)
    models, refs, nlls = [], [], []
    for b in range(B):
        preds, ev = O.ensemble_array(st[b])
        p = O.multicam_params(preds, ev, 0.01, 25)
        models.append(p)
        mf, Vf, S = O.filtering_pass(p["y"], p["m0"], p["S0"], p["C"], np.eye(n), p["A"], p["Q"], ev)
        ms, _, _ = O.smooth_backward(p["y"], mf, Vf, S, p["A"])
        refs.append(ms @ p["C"].T + p["means"])
        nlls.append(O.compute_nll(p["y"], p["m0"], p["S0"], p["C"], p["A"], p["Q"], ev))
    stk = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stk("m0"), stk("S0"), stk("A"), stk("Q"), stk("C"), stk("means"))
    d = batch.make_time_major(st, dtype=np.float64)
    res = batch.smooth(d, params, n=n, r=3, want_nll=True, check=True,
                       flags=batch.model_flags(stk("A"), stk("C")))
    assert np.abs(res["out"].cpu().numpy() - np.stack(refs)).max() < 1e-5
    np.testing.assert_allclose(res["nll"].cpu().numpy(), nlls, rtol=1e-9)
    np.testing.assert_allclose(batch.nll(d, params, n=n, r=3).cpu().numpy(), nlls, rtol=1e-9)


@pytest.mark.parametrize("r,n,B,T", [(3, 10, 3, 6000), (3, 12, 17, 3000), (3, 16, 2, 20000),
                                     (2, 2, 5, 4000), (3, 10, 1, 37)])
def test_runtime_n_time_parallel_equals_sequential(torch, rt_form, r, n, B, T):
    """The time-parallel runtime-n form (algo 2's chunk scans with the rows
    streamed) against the one-lane form: outputs, latent means and NLL
    (smoothing and filter-only calls), the tolerances of the compiled
    time-parallel algorithms (tests/test_gpu_configs.py PX_ALGO, NLL_RTOL);
    T = 20000 at B = 2 runs the wave-parallel chunk scans."""
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    rng = np.random.default_rng(n * 1000 + B)
    E = 5
    if r == 2:
        st = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3)
    else:
        st = synthetic.multiview_obs(rng, n // 2, E, T, K=B).transpose(2, 0, 1, 3)
    models = []
    for b in range(B):
        preds, ev = O.ensemble_array(st[b].astype(np.float64))
        models.append(O.singleview_params(preds, ev, 0.01, 25) if r == 2 else
                      O.multicam_params(preds, ev, 0.01, 25))
    stk = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stk("m0"), stk("S0"), stk("A"), stk("Q"), stk("C"), stk("means"))
    d = batch.make_time_major(st, dtype=np.float32)
    res = {}
    for form in (1, 2):
        rt_form(form)
        res[form] = batch.smooth(d, params, n=n, r=r, algo=4, flags=0, want_nll=True,
                                 want_ms=True, check=True)
        res[form]["nll_only"] = batch.nll(d, params, n=n, r=r, algo=4)
    a, b_ = res[1], res[2]
    assert float((a["out"] - b_["out"]).abs().max()) < 1e-8
    assert float((a["ms"] - b_["ms"]).abs().max()) < 1e-8
    for k in ("nll", "nll_only"):
        rel = float(((a[k] - b_[k]) / a[k].abs()).abs().max())
        assert rel < 1e-10, (k, rel)
    # and the oracle on the first trajectory
    p = models[0]
    ev = O.ensemble_array(st[0].astype(np.float64))[1]
    mf, Vf, S = O.filtering_pass(p["y"], p["m0"], p["S0"], p["C"], np.eye(n), p["A"], p["Q"], ev)
    ms, _, _ = O.smooth_backward(p["y"], mf, Vf, S, p["A"])
    ref = ms @ p["C"].T + p["means"]
    assert np.abs(b_["out"][0].cpu().numpy() - ref).max() < 1e-5


@pytest.mark.parametrize("V,E,dtype", [(5, 5, np.float32), (6, 4, np.float64), (8, 3, np.float32)])
def test_wide_fit_handoff_then_time_parallel_smooth(torch, V, E, dtype):
    """5-8 cameras end to end on the device: eks_fit (wide kernels) writes the
    y / ev hand-off planes, and the time-parallel runtime-n smoother reading
    them equals the same smoother reading the members, bit for bit (the same
    runtime-E ensemble either way)."""
    from eks_amd import batch, synthetic
    rng = np.random.default_rng(V * 10 + E)
    K, T, n = 3, 4000, 2 * V
    st = synthetic.multiview_obs(rng, V, E, T, K=K).astype(dtype)      # (E, T, K, n)
    obs = torch.from_numpy(np.ascontiguousarray(st.transpose(2, 1, 0, 3))).cuda()  # (K, T, E, n)
    params, _, yev = batch.fit(obs, kind="multicam", n=n, r=3, smooth_param=0.01,
                               quantile_keep=25, keep_yev=True)
    a = batch.smooth(obs, params, n=n, r=3, algo=4, want_nll=True, check=True)
    b = batch.smooth(yev, params, n=n, r=3, algo=4, want_nll=True, check=True)
    assert torch.equal(a["out"], b["out"])
    assert torch.equal(a["nll"], b["nll"])
    # the automatic choice (six cameras: the compiled r = 3, n = 12 kernels,
    # whose compile-time-E ensemble contracts differently) from the planes
    c = batch.smooth(yev, params, n=n, r=3, want_nll=True, check=True)
    assert float((c["out"] - a["out"]).abs().max()) < 1e-8
    torch.testing.assert_close(c["nll"], a["nll"], rtol=1e-10, atol=0)


def _multicam_batch(rng, V, E, B, T):
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    st = synthetic.multiview_obs(rng, V, E, T, K=B).transpose(2, 0, 1, 3)
    models = []
    for b in range(B):
        preds, ev = O.ensemble_array(st[b].astype(np.float64))
        models.append(O.multicam_params(preds, ev, 0.01, 25))
    stk = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stk("m0"), stk("S0"), stk("A"), stk("Q"), stk("C"), stk("means"))
    return st, params, batch.model_flags(stk("A"), stk("C"))


@pytest.mark.parametrize("n,B,T", [(12, 6, 3000), (12, 256, 400), (16, 4, 2500), (16, 264, 300)])
def test_compiled_wide_shapes_time_parallel_vs_sequential(torch, n, B, T):
    """Six- and eight-camera calls run compiled (r, n) = (3, 12) / (3, 16)
    kernels (eks_shape_312.hip / eks_shape_316.hip).  Explicit algo 2 and
    algo 3 from the member predictions -- few trajectories (group mode) and
    B >= 256 (whole-block chunks, k3_bwd's __launch_bounds__(256, 2)) --
    against algo 1: outputs, latent means and NLL at the compiled
    time-parallel tolerances (tests/test_gpu_configs.py PX_ALGO, NLL_RTOL)."""
    from eks_amd import batch
    rng = np.random.default_rng(n * 7 + B)
    st, params, flags = _multicam_batch(rng, n // 2, 5, B, T)
    d = batch.make_time_major(st, dtype=np.float32)
    ref = batch.smooth(d, params, n=n, r=3, algo=1, flags=flags, want_nll=True, want_ms=True,
                       check=True)
    for algo in (2, 3):
        res = batch.smooth(d, params, n=n, r=3, algo=algo, flags=flags, want_nll=True,
                           want_ms=True)
        assert int((res["status"] != 0).sum()) == 0, algo
        assert float((res["out"] - ref["out"]).abs().max()) < 1e-8, algo
        assert float((res["ms"] - ref["ms"]).abs().max()) < 1e-8, algo
        rel = float(((res["nll"] - ref["nll"]) / ref["nll"]).abs().max())
        assert rel < 1e-10, (algo, rel)


@pytest.mark.parametrize("n", [12, 16])
def test_compiled_wide_shapes_segmented(torch, n):
    """The phased time-shard path (eks_smooth_seg phases 1-3 + eks_seg_combine)
    at the compiled n = 12 / 16 shapes against the one-piece sequential call."""
    from eks_amd import batch, timeshard
    rng = np.random.default_rng(100 + n)
    st, params, flags = _multicam_batch(rng, n // 2, 5, 2, 6000)
    d = batch.make_time_major(st, dtype=np.float32)
    ref = batch.smooth(d, params, n=n, r=3, algo=1, flags=flags, want_nll=True, want_ms=True,
                       check=True)
    seg = timeshard.smooth_segments(d, params, n=n, r=3, nseg=3, flags=flags, want_ms=True)
    assert int((seg["status"] != 0).sum()) == 0
    assert float((seg["out"] - ref["out"]).abs().max()) < 1e-8
    assert float((seg["ms"] - ref["ms"]).abs().max()) < 1e-8
    np.testing.assert_allclose(seg["nll"].cpu().numpy(), ref["nll"].cpu().numpy(), rtol=1e-10)


def test_unsupported_shape_message_lists_compiled_shapes(torch):
    from eks_amd import _lib, batch
    rng = np.random.default_rng(3)
    st, params, flags = _multicam_batch(rng, 2, 3, 1, 50)
    d = batch.make_time_major(st, dtype=np.float32)
    # r = 4 has no kernels at all: the error lists the compiled shapes
    bad = torch.zeros((1, batch.param_len(4, 4)), dtype=torch.float64, device="cuda")
    with pytest.raises(_lib.EksError, match=r"\(3,12\) \(3,16\)"):
        batch.smooth(d, bad, n=4, r=4, algo=2, flags=0)
