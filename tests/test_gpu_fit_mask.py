"""eks_fit's kept-frame mask (k_fit_select -> k_fit_accum) against the
threshold path and the host fit.

With the ensemble hand-off planes requested (``keep_yev``), k_fit_select
also writes one bit per frame (worst ensemble variance <= the percentile
threshold, eks/multiview_pca_smoother.py:685-688) and k_fit_accum reads that
mask and the y plane instead of the ev plane.  The mask is built from three
sources -- frames below the threshold's top-digit bin (ballot in the
compaction pass), the bin's own frames (resolved in LDS against the
threshold), and a whole-row pass when the row is too long for the LDS mask,
the bin too large for the LDS candidates, or the threshold equals a key above
the bin -- and each must select exactly the frames ``v <= threshold`` does.
The check: the parameter rows of the mask path are bit-identical to those of
the member path (which compares v with the threshold itself), and both
match the host fit (numpy's percentile) to rounding.
"""
import warnings

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _fit_both(torch, st, q, n=2, r=2, kind="singleview"):
    """The member path and the mask path, each with both selection kernels
    (one block per row, and the split over row segments that few rows use):
    all four parameter sets bit-identical."""
    from eks_amd import _lib, batch
    obs = torch.from_numpy(np.ascontiguousarray(st)).cuda().permute(0, 2, 1, 3)  # (B,T,E,n)
    kw = dict(kind=kind, n=n, r=r, smooth_param=0.01, quantile_keep=q, check=False)
    res = []
    prev = _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, 1)
    try:
        for sel in (1, 2):
            _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, sel)
            p0, s0 = batch.fit(obs, **kw)
            p1, s1, _ = batch.fit(obs, keep_yev=True, **kw)
            res += [(p0.cpu().numpy(), s0.cpu().numpy()), (p1.cpu().numpy(), s1.cpu().numpy())]
    finally:
        _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, prev)
    p1 = res[1][0]
    for k, (p, st_) in enumerate(res):
        np.testing.assert_array_equal(st_, res[0][1])
        assert np.array_equal(p, p1, equal_nan=True), (k, np.nanmax(np.abs(p - p1)))
    return p1


def _vs_host(st, params, q):
    from eks_amd import fit
    from eks_amd.core import ensemble_array
    for b in range(st.shape[0]):
        preds, ev = ensemble_array(st[b].astype(np.float64))
        with np.errstate(all="ignore"), warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ref = fit.singleview_model(preds, ev, 0.01, q)
        got = params[b]
        want = np.concatenate([np.ravel(ref[k]) for k in ("m0", "S0", "A", "Q", "C", "offset")])
        scale = max(1.0, float(np.nanmax(np.abs(want))))
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-9 * scale, equal_nan=True)


@pytest.mark.parametrize("q", [0.0, 10.0, 25.0, 33.3, 50.0, 99.9, 100.0])
def test_mask_ties_quantised_members(torch, q):
    """Members on a 0.25 px grid: the worst variances take few distinct
    values, so the threshold's bin holds many ties and the threshold often
    equals a key exactly."""
    from eks_amd import synthetic
    rng = np.random.default_rng(int(q * 10) + 1)
    B, E, T = 8, 5, 3001
    st = np.stack([synthetic.singleview_obs(rng, E, T)[:, :, 0] for _ in range(B)])
    st = (np.round(st * 4.0) / 4.0).astype(np.float32)
    p = _fit_both(torch, st, q)
    _vs_host(st, p, q)


@pytest.mark.parametrize("T", [2, 63, 64, 65, 1000, 4000, 4097, 8010, 81000])
def test_mask_row_lengths(torch, T):
    """Rows shorter than a wave, exactly one word, ragged last words; and
    lengths where the last unrolled round of the selection's key loop ends
    inside a wave (T in (3840 + 4096 k, 4096 + 4096 k), T % 64 != 0 for the
    256-thread kernel: 4000, 8010; 81000 for the 1024-thread one): a wave
    split between the unrolled loop and the tail would ballot its mask word
    in two halves that overwrite each other (eks_fit.hip for_keys)."""
    from eks_amd import synthetic
    rng = np.random.default_rng(T)
    st = np.stack([synthetic.singleview_obs(rng, 3, T)[:, :, 0] for _ in range(5)])
    p = _fit_both(torch, st.astype(np.float64), 25.0)
    _vs_host(st, p, 25.0)


def test_mask_long_rows_whole_row_pass(torch):
    """T > 65 536 frames: no LDS mask (16-bit frame indices), the mask comes
    from the whole-row pass (and the 1024-thread select)."""
    from eks_amd import synthetic
    rng = np.random.default_rng(70001)
    st = np.stack([synthetic.singleview_obs(rng, 5, 70001)[:, :, 0] for _ in range(2)])
    p = _fit_both(torch, st, 25.0)
    _vs_host(st, p, 25.0)


@pytest.mark.parametrize("T,big,shift", [(16384, 1536, 50), (40000, 1536, 50),
                                         (400000, 19968, 49)])
def test_mask_bin_larger_than_lds(torch, T, big, shift):
    """No outliers and long rows: the threshold's top-digit bin holds more
    frames than the LDS candidate buffer (1 536 keys for one block per row
    with 13-bit digits -- at 16 384 frames the row still has its LDS mask, at
    40 000 not; 19 968 for the split selection's final block with 14-bit
    digits) in at least one row, so the select runs over the global row /
    candidate buffer and the mask comes from the whole-row pass."""
    from eks_amd import synthetic
    from eks_amd.core import ensemble_array
    rng = np.random.default_rng(20000 + T)
    q = 40.0
    st = np.stack([synthetic.singleview_obs(rng, 5, T, outlier_frac=0.0)[:, :, 0]
                   for _ in range(3)])
    counts = []
    for row in st:
        v = np.sort(ensemble_array(row.astype(np.float64))[1].max(axis=1))
        key = v.view(np.uint64) >> shift
        counts.append(int((key == key[int((T - 1) * q / 100)]).sum()))
    assert max(counts) > big, counts
    p = _fit_both(torch, st, q)
    _vs_host(st, p, q)


def test_mask_threshold_equals_key_above_bin(torch):
    """T = 2 and q just below 100: the threshold interpolates to within half
    an ulp of the larger key, which lies in a higher top-digit bin than the
    smaller one, so numpy keeps both frames; the LDS mask cannot see that
    frame and the select marks the row in a whole-row pass."""
    q = 99.99999999999999
    B, E = 4, 3
    st = np.zeros((B, E, 2, 2))
    for b in range(B):
        base = 100.0 + 10 * b
        st[b, :, 0, :] = base + np.array([-1.0, 0.0, 1.0])[:, None]          # var 2/9
        st[b, :, 1, :] = base + np.array([-1.0, 0.0, 1.0])[:, None] * (1.7, 2.3)[b % 2]
    from eks_amd.core import ensemble_array
    preds, ev = ensemble_array(st[0])
    v = ev.max(axis=1)
    thr = np.percentile(v, q)
    assert thr == v[1] and np.ptp(np.frombuffer(v.tobytes(), np.uint64) >> 51) > 0
    p = _fit_both(torch, st, q)
    _vs_host(st, p, q)


@pytest.mark.parametrize("q", [10.0, 25.0, 45.0])
@pytest.mark.parametrize("spread", [4, 40])
def test_mask_ties_below_32bit_resolution(torch, q, spread):
    """Worst variances that differ only in their low mantissa bits: members
    (-a, 0, a) with a = 1 + k 2^-23 (k < spread, exact in float32) give
    variances 2a^2/3 within ~1e-6 / 1e-5 relative, hundreds of frames per
    upper-32-bit key with distinct full keys, so every digit of the radix
    select and the mask's boundary frames are exercised on near-ties (a
    round-6 selection on 32-bit keys, measured and not kept, resolved these
    from the ev plane; profiles/r06/ab_fit/README.md).  The other half of
    the frames has a in [2, 3)."""
    rng = np.random.default_rng(int(q) * 7 + spread)
    B, E, T = 4, 3, 3000
    st = np.zeros((B, E, T, 2), np.float32)
    for b in range(B):
        a = (1.0 + rng.integers(0, spread, T) * 2.0 ** -23).astype(np.float32)
        big = rng.random(T) < 0.5
        a[big] = (2.0 + rng.random(big.sum())).astype(np.float32)
        st[b, 0, :, 0] = -a
        st[b, 2, :, 0] = a
        st[b, :, :, 1] = np.array([-0.5, 0.0, 0.5], np.float32)[:, None]  # smaller var
    from eks_amd.core import ensemble_array
    v = ensemble_array(st[0].astype(np.float64))[1].max(axis=1)
    hi32 = v.view(np.uint64) >> 32
    k = int((T - 1) * q / 100)
    tie = hi32 == (np.sort(v)[k:k + 1].view(np.uint64) >> 32)
    assert tie.sum() > 1 and np.unique(v[tie]).size > 1  # distinct full keys in one 32-bit key
    p = _fit_both(torch, st, q)
    _vs_host(st, p, q)


def test_mask_nan_row(torch):
    """A NaN member makes the row's percentile NaN: no frame kept, status
    reported, the same (NaN) parameters on both paths; other rows fit."""
    from eks_amd import synthetic
    rng = np.random.default_rng(9)
    st = np.stack([synthetic.singleview_obs(rng, 5, 800)[:, :, 0] for _ in range(4)])
    st[2, 1, 300, 0] = np.nan
    p = _fit_both(torch, st.astype(np.float32), 25.0)
    ok = [0, 1, 3]
    _vs_host(st[ok], p[ok], 25.0)


@pytest.mark.parametrize("V", [2, 4, 5, 8])
def test_mask_multicam(torch, V):
    from eks_amd import synthetic
    rng = np.random.default_rng(V)
    st = synthetic.multiview_obs(rng, V, 5, 2500, K=6).transpose(2, 0, 1, 3)
    _fit_both(torch, st, 25.0, n=2 * V, r=3, kind="multicam")
