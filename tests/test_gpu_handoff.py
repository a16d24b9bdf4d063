"""The per-keypoint wrappers smooth from the ensemble hand-off planes
(core.ensemble_handoff): one upload and one device reduction of the members
instead of two.  The planes must give the member path's result, and the
host copies must equal core.ensemble_array's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.mark.parametrize("mode", ["median", "mean"])
def test_handoff_singleview_equals_member_path(torch, mode):
    from eks_amd import core, fit, synthetic
    from eks_amd.smoothers import _run_fused
    rng = np.random.default_rng(11)
    stack = synthetic.singleview_obs(rng, 5, 3000)[:, :, 0].astype(np.float64)  # (E, T, 2)
    yev, preds, ev = core.ensemble_handoff(stack, mode)
    p2, e2 = core.ensemble_array(stack, mode)
    np.testing.assert_array_equal(preds, p2)
    np.testing.assert_array_equal(ev, e2)
    model = fit.singleview_model(preds, ev, 0.01, 25)
    a, _, nll_a = _run_fused(stack, model, mode=mode, want_nll=True)
    b, _, nll_b = _run_fused(stack, model, mode=mode, want_nll=True, yev=yev)
    np.testing.assert_allclose(b, a, rtol=0, atol=1e-10)
    assert abs(nll_a - nll_b) <= 1e-10 * abs(nll_a)


def test_handoff_multicam_equals_member_path(torch):
    from eks_amd import core, fit
    from eks_amd.smoothers import _run_fused
    rng = np.random.default_rng(12)
    E, T, V = 5, 2000, 4
    lat = np.cumsum(rng.normal(size=(T, 3)), axis=0)
    proj = rng.normal(size=(3, 2 * V))
    stack = lat @ proj + rng.normal(scale=0.5, size=(E, T, 2 * V))
    yev, preds, ev = core.ensemble_handoff(stack)
    model = fit.multicam_model(preds, ev, 0.01, 25)
    a, _, _ = _run_fused(stack, model)
    b, _, _ = _run_fused(stack, model, yev=yev)
    np.testing.assert_allclose(b, a, rtol=0, atol=1e-9)
