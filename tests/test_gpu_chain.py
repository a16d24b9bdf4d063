"""Robustness of the in-launch chains of the time-parallel passes.

algo 3's two persistent passes (two_pass.hpp) and algo 2's chained chunk
scans (smooth_impl.hpp) hand values between workgroups inside one launch;
every wait is bounded in wall-clock time (handoff.hpp) and a unit that gives
up flags its trajectories EKS_STATUS_SCAN.  These tests drive that path
(eks_debug_set(EKS_DBG_WAIT_US, -1): every wait gives up at once), check that
``batch.smooth(check=True)`` then re-runs the sequential kernel, check the
look-back chains' bit-reproducibility at the 8-GPU shard size, and force the
batch slicing of algo 3's member addressing (EKS_DBG_A3_SLICE_BYTES).
Reference recursion: eks/ensemble_kalman.py:59-164.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _singleview(torch, B, T, seed, E=5):
    from eks_amd import _lib, batch, synthetic
    rng = np.random.default_rng(seed)
    st = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float32)
    d = batch.make_time_major(st, dtype=np.float32)
    params = batch.fit(d, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)[0]
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    return d, params, flags


class _Forced:
    """every chain wait gives up at once while active"""

    def __enter__(self):
        from eks_amd import _lib
        self.prev = _lib.debug_set(_lib.EKS_DBG_WAIT_US, -1)
        return self

    def __exit__(self, *exc):
        from eks_amd import _lib
        _lib.debug_set(_lib.EKS_DBG_WAIT_US, self.prev if self.prev >= 0 else 0)


# algo 2: 3 trajectories x 400 000 frames -> 293 groups of chunks per
# trajectory, so the group-level chained scans run 2 blocks per trajectory
@pytest.mark.parametrize("algo,B,T", [(3, 130, 700), (2, 3, 400000)])
def test_forced_chain_timeout_flags_scan_and_check_reruns(torch, algo, B, T):
    """Every wait gives up: the launch still ends, the trajectories whose
    units had to wait carry EKS_STATUS_SCAN, and check=True re-runs them with
    algo 1, whose bits the result then has."""
    from eks_amd import _lib, batch
    d, params, flags = _singleview(torch, B, T, 7 + algo)
    ref = batch.smooth(d, params, n=2, r=2, algo=1, flags=flags, want_nll=True)
    with _Forced():
        bad = batch.smooth(d, params, n=2, r=2, algo=algo, flags=flags, want_nll=True)
        torch.cuda.synchronize()
        st = bad["status"].cpu().numpy()
        # (stale hand-off values may also trip other checks: only SCAN is promised)
        assert (st & _lib.EKS_STATUS_SCAN).all(), np.unique(st)
        good = batch.smooth(d, params, n=2, r=2, algo=algo, flags=flags, want_nll=True, check=True)
    assert (good["status"] == 0).all()
    assert torch.equal(good["out"], ref["out"])
    assert torch.equal(good["nll"], ref["nll"])
    if algo == 2:  # the filter-only call's chained scans (K2 with the NLL partials)
        with _Forced():
            stn = torch.empty((B,), dtype=torch.int32, device="cuda")
            batch.nll(d, params, n=2, r=2, algo=2, flags=flags, check=False, status=stn)
            assert (stn.cpu().numpy() & _lib.EKS_STATUS_SCAN).all()
    # the bound restored: the same call is clean again
    again = batch.smooth(d, params, n=2, r=2, algo=algo, flags=flags, want_nll=True)
    assert (again["status"] == 0).all()
    assert float((again["out"] - ref["out"]).abs().max()) < 1e-8


def test_debug_set_roundtrip():
    from eks_amd import _lib
    prev = _lib.debug_set(_lib.EKS_DBG_WAIT_US, 250000)
    assert prev == 1000000  # the default bound: 1 s
    assert _lib.debug_set(_lib.EKS_DBG_WAIT_US, 0) == 250000
    assert _lib.debug_set(_lib.EKS_DBG_A3_SLICE_BYTES, 0) == 0


def test_algo3_sliced_launches_bit_identical(torch):
    """The batch slicing of algo 3 (member byte offsets past the buffer
    descriptor's 4 GB range: consecutive slices on one stream and one
    workspace) forced with a small span: bit-identical to the one-piece
    call, including the ragged last slice, ms and NLL."""
    from eks_amd import _lib, batch
    B, T, E = 1000, 300, 5
    d, params, flags = _singleview(torch, B, T, 31, E)
    whole = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags, want_ms=True, want_nll=True)
    sb, st, se, sj = d.stride()
    soff = ((E - 1) * se + (2 - 1) * sj) * 4 + 4
    prev = _lib.debug_set(_lib.EKS_DBG_A3_SLICE_BYTES, soff + 384 * 4)  # 384 trajectories per slice
    try:
        sliced = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags, want_ms=True, want_nll=True)
    finally:
        _lib.debug_set(_lib.EKS_DBG_A3_SLICE_BYTES, prev)
    assert (sliced["status"] == 0).all()
    assert torch.equal(sliced["out"], whole["out"])
    assert torch.equal(sliced["ms"], whole["ms"])
    assert torch.equal(sliced["nll"], whole["nll"])


def test_algo3_shard_size_lookback_bit_identical(torch):
    """The 8-GPU shard of config 4 (128 videos = 2 176 trajectories, 10 000
    frames) is where the chains' look-back runs most (few groups per time
    chunk: units wait for neighbours still streaming).  The look-back folds
    published values with the sequential chain's own operations, so the
    shard's bits equal those of the same trajectories inside a larger batch
    (where almost every unit finds its neighbour's value ready) and of
    repeated calls; and they match the sequential recursion to 1e-8 px."""
    from eks_amd import _lib, batch
    B, T, E = 2 * 2176, 10000, 5
    g = torch.Generator(device="cuda")
    g.manual_seed(128)
    kw = dict(dtype=torch.float64, device="cuda", generator=g)
    lat = torch.rand((1, 1, 2, B), **kw) * 400 + torch.cumsum(torch.randn((T, 1, 2, B), **kw) * 2, 0)
    obs = (lat + torch.randn((T, E, 2, B), **kw) * (torch.rand((1, E, 1, B), **kw) * 2.5 + 0.5))
    d = obs.to(torch.float32).permute(3, 0, 1, 2)                  # (B, T, E, 2) view, time-major
    del lat, obs
    params = batch.fit(d, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)[0]
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    full = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags, want_nll=True)
    assert (full["status"] == 0).all()
    lo = 2176
    shard = [batch.smooth(d[lo:], params[lo:].contiguous(), n=2, r=2, algo=3, flags=flags,
                          want_nll=True) for _ in range(3)]
    for s in shard:
        assert (s["status"] == 0).all()
        assert torch.equal(s["out"], full["out"][lo:])
        assert torch.equal(s["nll"], full["nll"][lo:])
    ref = batch.smooth(d[lo:lo + 256], params[lo:lo + 256].contiguous(), n=2, r=2, algo=1,
                       flags=flags)
    assert float((shard[0]["out"][:256] - ref["out"]).abs().max()) < 1e-8


@pytest.mark.parametrize("B,T", [(700, 3000), (64, 1000), (2176, 2000)])
def test_algo3_lookback_forms_bit_identical(torch, B, T):
    """k3_bwd with and without its decoupled look-back (EKS_DBG_A3_LB 1 / 2):
    the same operations in the same association order, so the same bits
    (outputs, smoothed means, NLL); and the forced time-out flags every
    trajectory in both forms.  (Round 4's one-launch form of both passes was
    removed in round 5: it measured no better at any size.)"""
    from eks_amd import _lib, batch
    d, params, flags = _singleview(torch, B, T, 900 + B)
    runs = {}
    prev = _lib.debug_set(_lib.EKS_DBG_A3_LB, 1)
    try:
        for lb in (1, 2):
            _lib.debug_set(_lib.EKS_DBG_A3_LB, lb)
            runs[lb] = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags, want_ms=True,
                                    want_nll=True)
            assert (runs[lb]["status"] == 0).all(), lb
            with _Forced():
                bad = batch.smooth(d, params, n=2, r=2, algo=3, flags=flags)
                torch.cuda.synchronize()
                if T > 256:  # (more than one unit per trajectory: every unit but the first waits)
                    assert (bad["status"].cpu().numpy() & _lib.EKS_STATUS_SCAN).all()
    finally:
        _lib.debug_set(_lib.EKS_DBG_A3_LB, prev)
    for k in ("out", "ms", "nll"):
        assert torch.equal(runs[2][k], runs[1][k]), k


@pytest.mark.parametrize("algo,B,T", [(3, 2176, 2000), (2, 17, 100000)])
def test_chained_passes_repeat_bit_identical(torch, algo, B, T):
    """The in-launch hand-offs under repetition: 20 calls of the chained
    passes on one input (algo 3 at the 8-GPU shard's 34 trajectory groups,
    algo 2's chained group scans at config 2's geometry) all give the first
    call's bits, and that result matches algo 1 (no hand-offs) to rounding.
    tools/soak_handoff.py runs the same at 200 calls (profiles/r06/soak/)."""
    from eks_amd import batch
    d, params, flags = _singleview(torch, B, T, 31 + algo)
    ref = batch.smooth(d, params, n=2, r=2, algo=1, flags=flags, want_nll=True)
    first = batch.smooth(d, params, n=2, r=2, algo=algo, flags=flags, want_nll=True)
    assert (first["status"] == 0).all()
    assert float((first["out"] - ref["out"]).abs().max()) < 1e-8
    for _ in range(20):
        r = batch.smooth(d, params, n=2, r=2, algo=algo, flags=flags, want_nll=True)
        assert torch.equal(r["out"], first["out"]) and torch.equal(r["nll"], first["nll"])
        assert (r["status"] == 0).all()
