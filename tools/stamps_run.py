"""Phase breakdown of k3_bwd from in-kernel s_memtime stamps (experiment
build exp/stamps: exp/stamps.patch).  Runs config 4 (or --videos N) eagerly,
copies the stamps of the last call and prints mean cycles per phase."""
import ctypes as C
import os
import sys

import numpy as np

sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
from eks_amd import _lib  # noqa: E402

a = bench.parse()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
w = bench.workload_singleview(torch, a, dev, 0, 1, 4)
for _ in range(3):
    w["step"]()
torch.cuda.synchronize()
lib = _lib.load()
n = 512 * 128 * 32
buf = np.zeros(n, dtype=np.uint64)
lib.eks_dbg_stamps.restype = C.c_int
rc = lib.eks_dbg_stamps(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes))
assert rc == 0, rc
st = buf.reshape(512, 128, 4, 8).astype(np.int64)
names = ["fwd sweep", "bar1", "chain(w0)", "bar2", "bwd sweep", "bar3"]
rows = []
for blk in range(512):
    for it in range(128):
        s = st[blk, it]
        if s[0, 1] == 0:
            continue
        rows.append(s)
rows = np.array(rows)  # (units, 4 waves, 8)
print("units stamped", len(rows))
tot = rows[:, :, 7] - rows[:, :, 1]
for wv in range(4):
    d = [rows[:, wv, k + 1] - rows[:, wv, k] for k in range(1, 7)]
    print(f"wave {wv}: " + "  ".join(f"{nm}={np.mean(x):8.0f}" for nm, x in zip(names, d)) +
          f"  total={np.mean(tot[:, wv]):8.0f} cyc")
# gaps between units of one block (ticket decode, loop back)
gaps = []
for blk in range(512):
    s = st[blk]
    its = [i for i in range(128) if s[i, 0, 1] != 0]
    for i0, i1 in zip(its, its[1:]):
        gaps.append(s[i1, 0, 1] - s[i0, 0, 7])
print("gap between units (w0)", np.mean(gaps) if gaps else None)
# chain wait distribution (wave 0)
ch = rows[:, 0, 4] - rows[:, 0, 3]
print("chain w0 percentiles", np.percentile(ch, [10, 50, 90, 99]))
fw = rows[:, 0, 2] - rows[:, 0, 1]
print("fwd w0 percentiles", np.percentile(fw, [10, 50, 90, 99]))
