"""Phase breakdown of algo 3's passes from in-kernel s_memtime stamps
(profiling build: tools/build_cur.sh stamps -DEKS_STAMPS=1 eks_shape_22.hip,
then EKS_LIB=exp/stamps/libeks_hip.so).  Runs config 4 (or --videos N)
eagerly, copies the stamps of the last call and prints the mean cycles of
each phase per wave (two_pass.hpp EKS_STAMP points)."""
import ctypes as C
import os
import sys

import numpy as np

sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
from eks_amd import _lib  # noqa: E402

BLK, ITS = 512, 128
NAMES = {0: ["stream", "bar1", "chain(w0)", "bar2", "starts", "bar3"],
         1: ["fwd sweep", "bar1", "chain(w0)", "bar2", "bwd sweep", "bar3"]}

a = bench.parse()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
w = bench.workload_singleview(torch, a, dev, 0, 1, 4)
for _ in range(3):
    w["step"]()
torch.cuda.synchronize()
lib = _lib.load()
buf = np.zeros(2 * BLK * ITS * 32, dtype=np.uint64)
lib.eks_dbg_stamps.restype = C.c_int
assert lib.eks_dbg_stamps(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
st = buf.reshape(2, BLK, ITS, 4, 8).astype(np.int64)
for ps, kern in ((0, "k3_fwd"), (1, "k3_bwd")):
    rows = st[ps][st[ps][:, :, 0, 1] != 0]  # (units, 4 waves, 8)
    print(f"{kern}: units stamped {len(rows)}")
    if not len(rows):
        continue
    tot = rows[:, :, 7] - rows[:, :, 1]
    for wv in range(4):
        d = [rows[:, wv, k + 1] - rows[:, wv, k] for k in range(1, 7)]
        print(f"  wave {wv}: " + "  ".join(f"{nm}={np.mean(x):7.0f}" for nm, x in zip(NAMES[ps], d))
              + f"  total={np.mean(tot[:, wv]):7.0f} cyc")
    gaps = []
    for blk in range(BLK):
        s = st[ps, blk]
        its = [i for i in range(ITS) if s[i, 0, 1] != 0]
        gaps += [s[i1, 0, 1] - s[i0, 0, 7] for i0, i1 in zip(its, its[1:])]
    print("  gap between a block's units (w0):", np.percentile(gaps, [10, 50, 90]) if gaps else None)
    ch = rows[:, 0, 4] - rows[:, 0, 3]
    print("  chain w0 percentiles 10/50/90/99:", np.percentile(ch, [10, 50, 90, 99]))
    fw = rows[:, 0, 2] - rows[:, 0, 1]
    print("  first phase w0 percentiles 10/50/90/99:", np.percentile(fw, [10, 50, 90, 99]))
    # chain detail (EKS_STAMP_AUX): look-back end time in wave 1's slot 0,
    # units folded in wave 2's; rows without a look-back keep (group, chunk)
    tl, nf = rows[:, 1, 0], rows[:, 2, 0]
    ok = (tl > rows[:, 0, 3]) & (tl <= rows[:, 0, 4])
    if ok.any():
        wait, fold = tl[ok] - rows[ok, 0, 3], rows[ok, 0, 4] - tl[ok]
        print(f"  chain detail ({ok.sum()} of {len(rows)} units): wait mean {wait.mean():.0f} "
              f"p50 {np.median(wait):.0f} p90 {np.percentile(wait, 90):.0f}; rest (fold, publish) "
              f"mean {fold.mean():.0f} p50 {np.median(fold):.0f} p90 {np.percentile(fold, 90):.0f} cyc")
        n = nf[ok]
        for lo, hi in ((0, 0), (1, 3), (4, 7), (8, 15), (16, 63), (64, 1 << 30)):
            sel = (n >= lo) & (n <= hi)
            if sel.any():
                print(f"    folded {lo:>3}-{hi if hi < 1 << 30 else 'inf':>3}: {sel.sum():6d} units, "
                      f"wait {wait[sel].mean():7.0f}, rest {fold[sel].mean():7.0f} cyc")
