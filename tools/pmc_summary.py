"""Per-kernel averages of the counter CSVs tools/gpu_pmc.sh collects:
python tools/pmc_summary.py gpurun_out/pmc_TAG"""
import csv
import glob
import os
import sys
from collections import defaultdict

N_XCD, N_SIMD = 8, 256 * 4  # MI355X


def main(d):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for path in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
        per = defaultdict(float)  # (dispatch, kernel, counter) -> summed over dimensions
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?").split("(")[0].split("<")[0]
                key = (row.get("Dispatch_Id"), k, row.get("Counter_Name"))
                per[key] += float(row.get("Counter_Value", 0) or 0)
        for (disp, k, c), v in per.items():
            acc[k][c].append(v)
    for k in sorted(acc):
        print(k)
        for c in sorted(acc[k]):
            vals = acc[k][c]
            print(f"  {c:28s} mean {sum(vals) / len(vals):.6g}  (n={len(vals)})")
        cnt = {c: sum(v) / len(v) for c, v in acc[k].items()}
        if "SQ_WAVE_CYCLES" in cnt and "SQ_ACTIVE_INST_VALU" in cnt and cnt["SQ_WAVE_CYCLES"]:
            print(f"  VALU active / wave cycles    {cnt['SQ_ACTIVE_INST_VALU'] / cnt['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_WAIT_ANY" in cnt and cnt.get("SQ_WAVE_CYCLES"):
            print(f"  wait-any / wave cycles       {cnt['SQ_WAIT_ANY'] / cnt['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_WAVE_CYCLES" in cnt and cnt.get("GRBM_GUI_ACTIVE"):
            # SQ_WAVE_CYCLES counts quad-cycles, summed over every resident
            # wave; GRBM_GUI_ACTIVE is the sum over the 8 XCDs
            # (MI355X_MICROARCH.md, s_memtime vs SQ PMC units; DVFS
            # give-back): mean resident waves per SIMD over the dispatch =
            # 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) / (256 CUs * 4 SIMDs).
            # (SQ_LEVEL_WAVES / SQ_ACCUM_PREV_HIRES read 0 on gfx950.)
            occ = 4.0 * cnt["SQ_WAVE_CYCLES"] / (cnt["GRBM_GUI_ACTIVE"] / N_XCD) / N_SIMD
            print(f"  mean waves per SIMD          {occ:.3f}")
            if cnt.get("SQ_WAVES"):
                # a persistent grid keeps every wave resident for the whole
                # dispatch: SQ_WAVES / SIMDs is the launch-bounds figure
                print(f"  SQ_WAVES / SIMDs             {cnt['SQ_WAVES'] / N_SIMD:.3f}")

if __name__ == "__main__":
    main(sys.argv[1])
