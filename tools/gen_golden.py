"""Generate golden vectors by running the REFERENCE implementation.

Run in the build container only (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py

It imports ``/root/reference/eks`` (with an empty ``seaborn`` stand-in module
in ``sys.modules``: seaborn is imported by eks/newton_eks.py:8 but only used
for a plot at :59, and is not installed here), runs the reference functions on
seeded inputs and on the reference's own example data, and writes the inputs,
every intermediate and the outputs as ``.npz`` fixtures to ``tests/golden/``.
No reference source is copied; only numbers are written.  The fixtures are what
travels to the GPU box; the reference does not.
"""
from __future__ import annotations

import glob
import os
import sys
import types

import numpy as np
import pandas as pd

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, REPO)
from eks_amd import synthetic  # noqa: E402


def _import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
    sys.path.insert(0, REF)
    import eks.ensemble_kalman as ek  # noqa: F401
    import eks.multiview_pca_smoother as mv  # noqa: F401
    import eks.pupil_smoother as ps  # noqa: F401
    import eks.utils as ut  # noqa: F401
    return ek, mv, ps, ut


def _save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def _spd(rng, r, scale):
    M = rng.normal(size=(r, r))
    return scale * (M @ M.T / r + 0.5 * np.eye(r))


# -------------------------------------------------------------------------
def gen_core(ek):
    """filtering_pass / smooth_backward / kalman_dot on random systems."""
    cases = []
    for (r, n) in [(2, 2), (3, 4), (3, 6), (3, 8), (2, 5), (4, 8)]:
        for T in (1, 2, 3, 257):
            cases.append((r, n, T, "rand"))
    cases += [(2, 2, 1000, "rand"), (3, 8, 1000, "rand"), (2, 2, 300, "zero_var"),
              (3, 4, 300, "zero_var"), (3, 8, 300, "diagA"), (2, 2, 2000, "heavy")]
    for i, (r, n, T, kind) in enumerate(cases):
        rng = np.random.default_rng(1000 + i)
        A = np.eye(r) + 0.05 * rng.normal(size=(r, r))
        if kind == "diagA":
            A = np.diag(rng.uniform(0.95, 0.9999, size=r))
        Q = _spd(rng, r, 0.5)
        if kind == "heavy":
            A = np.eye(r)
            Q = _spd(rng, r, 1e-4)
        S0 = _spd(rng, r, 20.0)
        m0 = rng.normal(size=r)
        C = rng.normal(size=(n, r)) * 2.0
        x = np.cumsum(rng.normal(size=(T, r)), axis=0)
        y = x @ C.T + rng.normal(size=(T, n))
        ev = rng.uniform(0.05, 4.0, size=(T, n))
        if kind == "zero_var":
            # exact-agreement frames: one member-variance entry at zero in 20% of
            # frames (several zeros at once can make R + C P C^T singular, where
            # the reference's own answer is round-off noise)
            rows = np.where(rng.random(size=T) < 0.2)[0]
            ev[rows, rng.integers(0, n, size=len(rows))] = 0.0
        R_in = np.eye(n)
        R = R_in.copy()
        mf, Vf, S = ek.filtering_pass(y, m0, S0, C, R, A, Q, ev)
        if T >= 2:
            ms, Vs, CV = ek.smooth_backward(y, mf, Vf, S, A, Q, C)
        else:  # the reference's backward loop is empty for T == 1
            ms, Vs, CV = mf.copy(), Vf.copy(), np.zeros((0, r, r))
        vec = rng.normal(size=n)
        mat = rng.normal(size=(n, r))
        kd_vec = ek.kalman_dot(vec, S0, C, np.diag(ev[0]))
        kd_mat = ek.kalman_dot(mat, S0, C, np.diag(ev[0]))
        _save(f"core_{kind}_r{r}_n{n}_T{T}", y=y, m0=m0, S0=S0, C=C, R_in=R_in, A=A, Q=Q,
              ev=ev, mf=mf, Vf=Vf, S=S, ms=ms, Vs=Vs, CV=CV, R_out=R,
              kd_vec_in=vec, kd_mat_in=mat, kd_vec=kd_vec, kd_mat=kd_mat)


def gen_ensemble(ek):
    """ensemble() on member stacks, both modes, odd/even E, with NaNs."""
    for E in (1, 2, 3, 4, 5, 8):
        for mode in ("median", "mean"):
            rng = np.random.default_rng(50 + E)
            T, n = 64, 3
            stack = rng.normal(100.0, 20.0, size=(E, T, n))
            if E == 5:
                stack[2, 7, 1] = np.nan
            keys = [f"kp{j}" for j in range(n)]
            dfs = [pd.DataFrame(stack[e], columns=keys) for e in range(E)]
            preds, var, stacks, _, _, _ = ek.ensemble(dfs, keys, mode=mode)
            _save(f"ensemble_E{E}_{mode}", stack=stack, preds=preds, vars=var, stacks=stacks)


SINGLEVIEW_CASES = {"c1": (3, 1000, 0, 0.01, 25.0), "c2small": (5, 3000, 2, 0.01, 25.0),
                    "q100": (4, 500, 7, 0.5, 100.0),
                    # members on a 0.25 px grid (float32-exact): the worst
                    # variances take few distinct values, so the percentile
                    # threshold ties with many frames -- pins which frames the
                    # reference keeps (its var / E arithmetic) at E = 3 and 5
                    "quant3": (3, 2000, 11, 0.01, 25.0), "quant5": (5, 2000, 12, 0.01, 40.0)}


def gen_singleview(ek, only=None):
    """Single-view definition computed with the reference's
    ensemble/filtering_pass/smooth_backward."""
    for name, (E, T, seed, s, q) in SINGLEVIEW_CASES.items():
        if only and name not in only:
            continue
        rng = np.random.default_rng(seed)
        obs = synthetic.singleview_obs(rng, E, T, K=1)[:, :, 0, :].astype(np.float64)
        if name.startswith("quant"):
            obs = np.round(obs * 4.0) / 4.0
        keys = ["kp_x", "kp_y"]
        dfs = [pd.DataFrame(obs[e], columns=keys) for e in range(E)]
        preds, ev, _, _, _, _ = ek.ensemble(dfs, keys)
        max_vars = np.max(ev, 1)
        good = np.where(max_vars <= np.percentile(max_vars, q))[0]
        means = preds[good].mean(axis=0)
        y = preds - means
        gy = y[good]
        m0 = np.zeros(2)
        S0 = np.diag(np.var(gy, axis=0))
        A = np.eye(2)
        C = np.eye(2)
        Q = s * np.cov((gy[1:] - gy[:-1]).T)
        R = np.eye(2)
        mf, Vf, S = ek.filtering_pass(y, m0, S0, C, R, A, Q, ev)
        ms, Vs, _ = ek.smooth_backward(y, mf, Vf, S, A, Q, C)
        out = (C @ ms.T).T + means
        _save(f"singleview_{name}", obs=obs, s=s, q=q, preds=preds, ev=ev, means=means,
              m0=m0, S0=S0, A=A, C=C, Q=Q, mf=mf, Vf=Vf, S=S, ms=ms, Vs=Vs, out=out,
              good=good)


def _mouse_markers(ut):
    files = sorted(glob.glob(os.path.join(REF, "data/mirror-mouse/*.csv")))
    markers = []
    for f in files:
        df = pd.read_csv(f, header=[0, 1, 2], index_col=0)
        kps = [c[1] for c in df.columns[::3]]
        markers.append(ut.convert_lp_dlc(df, kps, model_name=df.columns[0][0]))
    return markers


def gen_multicam(mv, ut):
    """mirror-mouse: reference pipeline (s=.01, q=25) for one paw, full T, plus
    the committed golden eks.csv columns for that paw."""
    markers = _mouse_markers(ut)
    cams = ["top", "bot"]
    golden = pd.read_csv(os.path.join(REF, "data/mirror-mouse/output/eks.csv"),
                         header=[0, 1, 2], index_col=0)
    for paw in ("paw2LF", "paw4RH"):
        by_cam = [[] for _ in cams]
        stacks = []
        for c, cam in enumerate(cams):
            cols = [f"{paw}_{cam}_x", f"{paw}_{cam}_y"]
            for m in markers:
                by_cam[c].append(m[cols])
            stacks.append(np.stack([m[cols].to_numpy() for m in markers]))  # (E,T,2)
        dfs = mv.ensemble_kalman_smoother_multi_cam(by_cam, paw, 0.01, 25, cams)
        out = np.concatenate(
            [dfs[f"{cam}_df"].loc[:, ("ensemble-kalman_tracker", paw, c)].to_numpy()[:, None]
             for cam in cams for c in ("x", "y")], axis=1)
        gold = np.concatenate(
            [golden.loc[:, ("ensemble-kalman_tracker", f"{paw}_{cam}", c)].to_numpy()[:, None]
             for cam in cams for c in ("x", "y")], axis=1)
        print(f"  {paw}: reference re-run vs committed golden max|d| = {np.abs(out - gold).max():.2e}")
        _save(f"multicam_mouse_{paw}", stacks=np.stack(stacks), s=0.01, q=25.0, out=out, golden=gold)


def gen_fish(ut, mv):
    """mirror-fish clips (3 cams, T=51, s=.01, q=50) vs the committed
    test_script.py outputs in data/misc/mirror-fish_ensemble-predictions/eks."""
    base = os.path.join(REF, "data/misc/mirror-fish_ensemble-predictions")
    cams = ["main", "top", "right"]
    tracker = "heatmap_mhcrnn_tracker"
    clips = [("20210126_Sean", "img001058.csv"), ("20210202_Quin", None)]
    for session, frame in clips:
        if frame is None:
            frame = sorted(os.listdir(os.path.join(base, "network_0", session)))[0]
        markers = []
        for k in range(5):
            df = pd.read_csv(os.path.join(base, f"network_{k}", session, frame), header=[0, 1, 2],
                             index_col=0)
            kps = [c[1] for c in df.columns[::3]]
            markers.append(ut.convert_lp_dlc(df, kps, model_name=tracker))
        golden = pd.read_csv(os.path.join(base, "eks", session, frame), header=[0, 1, 2], index_col=0)
        for kp in ("head", "mid"):
            stacks, by_cam = [], [[] for _ in cams]
            for c, cam in enumerate(cams):
                cols = [k for k in markers[0].keys() if cam in k and "likelihood" not in k and kp in k]
                for m in markers:
                    by_cam[c].append(m[cols])
                stacks.append(np.stack([m[cols].to_numpy() for m in markers]))
            dfs = mv.ensemble_kalman_smoother_multi_cam(by_cam, kp, 0.01, 50, cams)
            out = np.concatenate(
                [dfs[f"{cam}_df"].loc[:, ("ensemble-kalman_tracker", kp, c)].to_numpy()[:, None]
                 for cam in cams for c in ("x", "y")], axis=1)
            gold = np.concatenate(
                [golden.loc[:, (tracker, f"{kp}_{cam}", c)].to_numpy()[:, None]
                 for cam in cams for c in ("x", "y")], axis=1)
            print(f"  fish {session}/{frame}/{kp}: re-run vs golden max|d| = {np.abs(out - gold).max():.2e}")
            _save(f"multicam_fish_{session}_{kp}", stacks=np.stack(stacks), s=0.01, q=50.0,
                  out=out, golden=gold)


def gen_pupil(ps, ut):
    """ibl-pupil with A = diag(.99,.99,.99) (scripts/readme.txt:7) vs the committed
    golden kalman_smoothed_*.csv."""
    files = sorted(glob.glob(os.path.join(REF, "data/ibl-pupil/*.csv")))
    markers = []
    for f in files:
        df = pd.read_csv(f, header=[0, 1, 2], index_col=0)
        kps = [c[1] for c in df.columns[::3]]
        markers.append(ut.convert_lp_dlc(df, kps, model_name=df.columns[0][0]))
    A = np.diag([0.99, 0.99, 0.99])
    res = ps.ensemble_kalman_smoother_pupil(markers, kps, "ensemble-kalman_tracker", A)
    keys = ['pupil_top_r_x', 'pupil_top_r_y', 'pupil_bottom_r_x', 'pupil_bottom_r_y',
            'pupil_right_r_x', 'pupil_right_r_y', 'pupil_left_r_x', 'pupil_left_r_y']
    stack = np.stack([m[keys].to_numpy() for m in markers])
    mk = res["markers_df"].to_numpy()
    lat = res["latents_df"].to_numpy()
    g_mk = pd.read_csv(os.path.join(REF, "data/misc/pupil-test/kalman_smoothed_pupil_traces.csv"),
                       header=[0, 1, 2], index_col=0).to_numpy()
    g_lat = pd.read_csv(os.path.join(REF, "data/misc/pupil-test/kalman_smoothed_latents.csv"),
                        header=[0, 1], index_col=0).to_numpy()
    print(f"  pupil: markers re-run vs golden {np.nanmax(np.abs(mk - g_mk)):.2e}, "
          f"latents {np.abs(lat - g_lat).max():.2e}")
    _save("pupil_ibl", stack=stack, A=A, markers=mk, latents=lat, golden_markers=g_mk,
          golden_latents=g_lat, keypoint_names=np.array(kps))


def gen_newton(mv, ps, ut):
    """kalman_newton_recursive (eks/newton_eks.py:115) on random systems, the
    mirror-mouse opti golden (eks_opti.csv) and the pupil opti golden."""
    import eks.newton_eks as ne
    for i, (r, n, T, it) in enumerate([(2, 2, 1, 1), (2, 2, 2, 1), (3, 4, 200, 1), (3, 8, 300, 1),
                                       (2, 2, 300, 3), (3, 6, 100, 2)]):
        rng = np.random.default_rng(3000 + i)
        A = np.eye(r) + 0.05 * rng.normal(size=(r, r))
        E = _spd(rng, r, 0.5)
        S0 = _spd(rng, r, 20.0)
        mu0 = rng.normal(size=r)
        B = rng.normal(size=(n, r)) * 2.0
        x = np.cumsum(rng.normal(size=(T, r)), axis=0)
        y = x @ B.T + rng.normal(size=(T, n))
        ev = rng.uniform(0.05, 4.0, size=(T, n))
        res = ne.kalman_newton_recursive(y, mu0, S0, A, B, ev, E, max_iter=it)
        q = res if it == 1 else res[0]
        _save(f"newton_r{r}_n{n}_T{T}_it{it}", y=y, mu0=mu0, S0=S0, A=A, B=B, ev=ev, E=E,
              max_iter=it, q=q)
    # mirror-mouse opti golden: eks_opti_smoother_multi_cam(..., 0.01, 25, plot=False)
    markers = _mouse_markers(ut)
    cams = ["top", "bot"]
    golden = pd.read_csv(os.path.join(REF, "data/mirror-mouse/output/eks_opti.csv"),
                         header=[0, 1, 2], index_col=0)
    for paw in ("paw2LF",):
        by_cam, stacks = [[] for _ in cams], []
        for c, cam in enumerate(cams):
            cols = [f"{paw}_{cam}_x", f"{paw}_{cam}_y"]
            for m in markers:
                by_cam[c].append(m[cols])
            stacks.append(np.stack([m[cols].to_numpy() for m in markers]))
        dfs = mv.eks_opti_smoother_multi_cam(by_cam, paw, 0.01, 25, cams, plot=False)
        out = np.concatenate(
            [dfs[f"{cam}_df"].loc[:, ("ensemble-kalman_tracker", paw, c)].to_numpy()[:, None]
             for cam in cams for c in ("x", "y")], axis=1)
        gold = np.concatenate(
            [golden.loc[:, ("ensemble-kalman_tracker", f"{paw}_{cam}", c)].to_numpy()[:, None]
             for cam in cams for c in ("x", "y")], axis=1)
        print(f"  opti {paw}: re-run vs committed golden max|d| = {np.abs(out - gold).max():.2e}")
        _save(f"opti_mouse_{paw}", stacks=np.stack(stacks), s=0.01, q=25.0, out=out, golden=gold)
    # pupil opti golden: the Newton filter with the pupil model and A = 0.99 I
    # (eks/pupil_smoother.py:227-320), committed as data/misc/pupil-test/opti_eks_latents.csv
    files = sorted(glob.glob(os.path.join(REF, "data/ibl-pupil/*.csv")))
    mk = []
    for f in files:
        df = pd.read_csv(f, header=[0, 1, 2], index_col=0)
        kps = [c[1] for c in df.columns[::3]]
        mk.append(ut.convert_lp_dlc(df, kps, model_name=df.columns[0][0]))
    keys = ['pupil_top_r_x', 'pupil_top_r_y', 'pupil_bottom_r_x', 'pupil_bottom_r_y',
            'pupil_right_r_x', 'pupil_right_r_y', 'pupil_left_r_x', 'pupil_left_r_y']
    import eks.ensemble_kalman as ek
    preds, ev, _, avg_d, _, _ = ek.ensemble(mk, keys)
    loc = ps.get_pupil_location(avg_d)
    diam = ps.get_pupil_diameter(avg_d)
    mx, my = loc[:, 0].mean(), loc[:, 1].mean()
    y = preds.copy()
    y[:, 0::2] -= mx
    y[:, 1::2] -= my
    A = np.diag([0.99, 0.99, 0.99])
    mu0 = np.array([diam.mean(), 0.0, 0.0])
    vx, vy = np.var(loc[:, 0] - mx), np.var(loc[:, 1] - my)
    S0 = np.diag([np.var(diam), vx, vy])
    E = np.diag([np.var(diam) * (1 - 0.99 ** 2), vx * (1 - 0.99 ** 2), vy * (1 - 0.99 ** 2)])
    B = np.array([[0, 1, 0], [-.5, 0, 1], [0, 1, 0], [.5, 0, 1], [.5, 1, 0], [0, 0, 1],
                  [-.5, 1, 0], [0, 0, 1]], dtype=np.float64)
    q = ne.kalman_newton_recursive(y, mu0, S0, A, B, ev, E)
    lat = np.stack([q[:, 0], q[:, 1] + mx, q[:, 2] + my], 1)
    g = pd.read_csv(os.path.join(REF, "data/misc/pupil-test/opti_eks_latents.csv"),
                    header=[0, 1], index_col=0).to_numpy()
    print(f"  opti pupil latents vs committed golden max|d| = {np.abs(lat - g).max():.2e}")
    _save("opti_pupil_ibl", stack=np.stack([m[keys].to_numpy() for m in mk]), A=A, latents=lat,
          golden_latents=g)


def gen_cli(mv, ps, ut):
    """Script-level fixtures (F1): the first 300 frames of the mirror-mouse and
    ibl-pupil member CSVs (data lines copied verbatim) and the outputs the
    reference's scripts produce on them (scripts/multicam_example.py,
    scripts/pupil_example.py), with the reference functions the scripts call."""
    import eks.newton_eks as ne
    import eks.ensemble_kalman as ek
    nrow = 300
    base = os.path.join(OUT, "csv")
    for ds in ("mirror-mouse", "ibl-pupil"):
        os.makedirs(os.path.join(base, ds), exist_ok=True)
        for f in sorted(glob.glob(os.path.join(REF, "data", ds, "*.csv"))):
            lines = open(f).read().splitlines(True)
            with open(os.path.join(base, ds, os.path.basename(f)), "w") as fo:
                fo.writelines(lines[:3 + nrow])
    exp = os.path.join(base, "expected")
    os.makedirs(exp, exist_ok=True)

    def load(ds):
        ml, raw = [], None
        for f in sorted(glob.glob(os.path.join(base, ds, "*.csv"))):
            raw = pd.read_csv(f, header=[0, 1, 2], index_col=0)
            kps = [c[1] for c in raw.columns[::3]]
            ml.append(ut.convert_lp_dlc(raw, kps, model_name=raw.columns[0][0]))
        return ml, raw, kps

    # multicam_example.py (:96-160), both eks versions
    ml, raw, _ = load("mirror-mouse")
    cams = ["top", "bot"]
    for version, fn, fname in (("standard", mv.ensemble_kalman_smoother_multi_cam, "eks.csv"),
                               ("opti", mv.eks_opti_smoother_multi_cam, "eks_opti.csv")):
        out = raw.copy()
        out.columns = out.columns.set_levels(['ensemble-kalman_tracker'], level=0)
        for col in out.columns:
            out[col].values[:] = 1.0 if col[-1] == 'likelihood' else np.nan
        for kp in ["paw1LH", "paw2LF", "paw3RF", "paw4RH"]:
            by_cam = [[] for _ in cams]
            for m in ml:
                for c, cam in enumerate(cams):
                    keys = [k for k in m.keys() if cam in k and 'likelihood' not in k and kp in k]
                    by_cam[c].append(m[keys])
            kw = dict(plot=False) if version == "opti" else {}
            dfs = fn(by_cam, kp, 0.01, 25, cams, **kw)
            for cam in cams:
                for coord in ("x", "y"):
                    out.loc[:, ('ensemble-kalman_tracker', f'{kp}_{cam}', coord)] = \
                        dfs[f'{cam}_df'].loc[:, ('ensemble-kalman_tracker', kp, coord)]
        out.to_csv(os.path.join(exp, fname))
        print(f"  wrote expected/{fname}")
    # pupil_example.py (:76-114), --diameter-s .99 --com-s .99
    ml, raw, kps = load("ibl-pupil")
    A = np.diag([0.99, 0.99, 0.99])
    d = ps.ensemble_kalman_smoother_pupil(ml, kps, 'ensemble-kalman_tracker', A)
    d['markers_df'].to_csv(os.path.join(exp, "kalman_smoothed_pupil_traces.csv"))
    d['latents_df'].to_csv(os.path.join(exp, "kalman_smoothed_latents.csv"))
    # opti: eks_opti_smoother_pupil's computation (its plot=False branch
    # references an undefined q; see eks_amd.smoothers.eks_opti_smoother_pupil)
    keys = ['pupil_top_r_x', 'pupil_top_r_y', 'pupil_bottom_r_x', 'pupil_bottom_r_y',
            'pupil_right_r_x', 'pupil_right_r_y', 'pupil_left_r_x', 'pupil_left_r_y']
    preds, ev, _, avg_d, _, _ = ek.ensemble(ml, keys)
    loc = ps.get_pupil_location(avg_d)
    diam = ps.get_pupil_diameter(avg_d)
    mx, my = loc[:, 0].mean(), loc[:, 1].mean()
    y = preds.copy()
    y[:, 0::2] -= mx
    y[:, 1::2] -= my
    vx, vy, vd = np.var(loc[:, 0] - mx), np.var(loc[:, 1] - my), np.var(diam)
    Bm = np.array([[0, 1, 0], [-.5, 0, 1], [0, 1, 0], [.5, 0, 1], [.5, 1, 0], [0, 0, 1],
                   [-.5, 1, 0], [0, 0, 1]], dtype=np.float64)
    q = ne.kalman_newton_recursive(y, np.array([diam.mean(), 0.0, 0.0]), np.diag([vd, vx, vy]), A,
                                   Bm, ev, np.diag([vd, vx, vy]) * (1 - 0.99 ** 2))
    mk = q @ Bm.T
    mk[:, 0::2] += mx
    mk[:, 1::2] += my
    nan = np.full(len(q), np.nan)
    cols = []
    for kp in ('top', 'right', 'bottom', 'left'):
        j = keys.index(f'pupil_{kp}_r_x')
        cols += [mk[:, j], mk[:, j + 1], nan]
    pd.DataFrame(np.stack(cols, 1), columns=ut.make_dlc_pandas_index(kps)).to_csv(
        os.path.join(exp, "opti_eks_pupil_traces.csv"))
    idx = pd.MultiIndex.from_arrays([['ensemble-kalman_tracker'] * 3,
                                     ['diameter', 'com_x', 'com_y']], names=('scorer', 'latent'))
    pd.DataFrame(np.stack([q[:, 0], q[:, 1] + mx, q[:, 2] + my], 1), columns=idx).to_csv(
        os.path.join(exp, "opti_eks_latents.csv"))
    print("  wrote expected pupil outputs")


def gen_paw(mv, ut):
    """ibl-paw (F4): the first 300 left-camera frames and the right-camera
    frames spanning them, both eks versions of the asynchronous paw smoother
    on them (eks/multiview_pca_smoother.py:34, :325), loaded as the
    reference's scripts/multiview_paw_example.py:66-97 does (right-camera paws
    swapped).  Timestamps read with numpy.load(allow_pickle=False)."""
    src = os.path.join(REF, "data", "ibl-paw")
    base = os.path.join(OUT, "csv", "ibl-paw")
    os.makedirs(base, exist_ok=True)
    stem = "3f859b5c-e73a-4044-b49e-34bb81e96715"
    tl = np.load(os.path.join(src, f"{stem}.timestamps.left.npy"))
    tr = np.load(os.path.join(src, f"{stem}.timestamps.right.npy"))
    nl = 300
    nr = int(np.searchsorted(tr, tl[nl - 1], side="right")) + 2
    np.save(os.path.join(base, f"{stem}.timestamps.left.npy"), tl[:nl])
    np.save(os.path.join(base, f"{stem}.timestamps.right.npy"), tr[:nr])
    for f in sorted(glob.glob(os.path.join(src, "*.csv"))):
        n = nl if ".left." in f else nr
        lines = open(f).read().splitlines(True)
        with open(os.path.join(base, os.path.basename(f)), "w") as fo:
            fo.writelines(lines[:3 + n])
    left, right = [], []
    for f in sorted(glob.glob(os.path.join(base, "*.csv"))):
        raw = pd.read_csv(f, header=[0, 1, 2], index_col=0)
        kps = [c[1] for c in raw.columns[::3]]
        fmt = ut.convert_lp_dlc(raw, kps, model_name=raw.columns[0][0])
        if "left" in os.path.basename(f):
            left.append(fmt)
        else:
            cols = {'paw_l_x': 'paw_r_x', 'paw_l_y': 'paw_r_y', 'paw_l_likelihood': 'paw_r_likelihood',
                    'paw_r_x': 'paw_l_x', 'paw_r_y': 'paw_l_y', 'paw_r_likelihood': 'paw_l_likelihood'}
            fmt = fmt.rename(columns=cols).loc[:, list(cols.keys())]
            right.append(fmt)
    exp = os.path.join(OUT, "csv", "expected")
    os.makedirs(exp, exist_ok=True)
    tl_, tr_ = tl[:nl], tr[:nr]
    res = {}
    for name, fn in (("standard", mv.ensemble_kalman_smoother_paw_asynchronous),
                     ("opti", mv.eks_opti_smoother_paw_asynchronous)):
        d = fn(left, right, tl_, tr_, kps, 1.0, 25)
        prefix = "eks_opti" if name == "opti" else "kalman"
        for view in ("left", "right"):
            d[f"{view}_df"].to_csv(os.path.join(exp, f"{prefix}_smoothed_paw_traces.{view}.csv"))
        res[name] = d
    _save("paw_async",
          left=np.stack([m.to_numpy() for m in left]), right=np.stack([m.to_numpy() for m in right]),
          tl=tl_, tr=tr_, s=1.0, q=25.0,
          **{f"{k}_{v}": res[k][f"{v}_df"].to_numpy() for k in res for v in ("left", "right")})
    print("  wrote paw fixtures")


def gen_bign(ek, mv):
    """Observation dimensions above the compiled kernels' n <= 8 (5 and 6
    cameras: n = 10, 12): filtering_pass / smooth_backward / kalman_dot, the
    Newton filter, and eks_opti_smoother_multi_cam on 5 synthetic cameras."""
    import eks.newton_eks as ne
    cases = [(3, 10, 3, "rand"), (3, 10, 257, "rand"), (3, 12, 257, "rand"),
             (3, 10, 300, "zero_var")]
    for i, (r, n, T, kind) in enumerate(cases):
        rng = np.random.default_rng(5000 + i)
        A = np.eye(r) + 0.05 * rng.normal(size=(r, r))
        Q = _spd(rng, r, 0.5)
        S0 = _spd(rng, r, 20.0)
        m0 = rng.normal(size=r)
        C = rng.normal(size=(n, r)) * 2.0
        x = np.cumsum(rng.normal(size=(T, r)), axis=0)
        y = x @ C.T + rng.normal(size=(T, n))
        ev = rng.uniform(0.05, 4.0, size=(T, n))
        if kind == "zero_var":
            rows = np.where(rng.random(size=T) < 0.2)[0]
            ev[rows, rng.integers(0, n, size=len(rows))] = 0.0
        R_in = np.eye(n)
        R = R_in.copy()
        mf, Vf, S = ek.filtering_pass(y, m0, S0, C, R, A, Q, ev)
        ms, Vs, CV = ek.smooth_backward(y, mf, Vf, S, A, Q, C)
        vec = rng.normal(size=n)
        mat = rng.normal(size=(n, r))
        kd_vec = ek.kalman_dot(vec, S0, C, np.diag(ev[0]))
        kd_mat = ek.kalman_dot(mat, S0, C, np.diag(ev[0]))
        _save(f"core_{kind}_r{r}_n{n}_T{T}", y=y, m0=m0, S0=S0, C=C, R_in=R_in, A=A, Q=Q,
              ev=ev, mf=mf, Vf=Vf, S=S, ms=ms, Vs=Vs, CV=CV, R_out=R,
              kd_vec_in=vec, kd_mat_in=mat, kd_vec=kd_vec, kd_mat=kd_mat)
    for i, (r, n, T, it) in enumerate([(3, 10, 200, 1), (3, 12, 100, 2)]):
        rng = np.random.default_rng(6000 + i)
        A = np.eye(r) + 0.05 * rng.normal(size=(r, r))
        E = _spd(rng, r, 0.5)
        S0 = _spd(rng, r, 20.0)
        mu0 = rng.normal(size=r)
        B = rng.normal(size=(n, r)) * 2.0
        x = np.cumsum(rng.normal(size=(T, r)), axis=0)
        y = x @ B.T + rng.normal(size=(T, n))
        ev = rng.uniform(0.05, 4.0, size=(T, n))
        res = ne.kalman_newton_recursive(y, mu0, S0, A, B, ev, E, max_iter=it)
        q = res if it == 1 else res[0]
        _save(f"newton_r{r}_n{n}_T{T}_it{it}", y=y, mu0=mu0, S0=S0, A=A, B=B, ev=ev, E=E,
              max_iter=it, q=q)
    # eks_opti_smoother_multi_cam with V = 5 cameras (n = 10), E = 4 members
    V, E, T = 5, 4, 300
    st = synthetic.multiview_obs(np.random.default_rng(6100), V, E, T, K=1)[:, :, 0, :]
    st = st.astype(np.float64)                                   # (E, T, 2V)
    cams = [f"cam{c}" for c in range(V)]
    kp = "paw"
    by_cam = [[pd.DataFrame(st[e][:, 2 * c:2 * c + 2], columns=[f"{kp}_x", f"{kp}_y"])
               for e in range(E)] for c in range(V)]
    dfs = mv.eks_opti_smoother_multi_cam(by_cam, kp, 0.01, 25, cams, plot=False)
    out = np.concatenate(
        [dfs[f"{cam}_df"].loc[:, ("ensemble-kalman_tracker", kp, c)].to_numpy()[:, None]
         for cam in cams for c in ("x", "y")], axis=1)
    _save("opti_multicam_V5", stack=st, s=0.01, q=25.0, out=out)


def main():
    ek, mv, ps, ut = _import_reference()
    if len(sys.argv) > 1 and sys.argv[1] == "bign":
        gen_bign(ek, mv)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "paw":
        gen_paw(mv, ut)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "cli":
        gen_cli(mv, ps, ut)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "quant":
        gen_singleview(ek, only=("quant3", "quant5"))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "newton":
        gen_newton(mv, ps, ut)
        return
    gen_core(ek)
    gen_ensemble(ek)
    gen_singleview(ek)
    gen_multicam(mv, ut)
    gen_fish(ut, mv)
    gen_pupil(ps, ut)
    gen_newton(mv, ps, ut)
    gen_cli(mv, ps, ut)
    gen_paw(mv, ut)
    gen_bign(ek, mv)


if __name__ == "__main__":
    main()
