"""Summarise a tools/gpu_profile.sh run into profiles/<tag>/.

    python tools/prof_summary.py gpurun_out/prof_r01 profiles/r01 [workload_key, e.g. config4-singleview-v1024-k17-e5-t10000-a3]

Reads the rocprofv3 kernel-stats CSV and the FETCH_SIZE / WRITE_SIZE counter
CSVs (separate passes), keeps the EKS kernels, and writes
  profiles/<tag>/kernel_stats.csv      (copied rocprofv3 --stats summary)
  profiles/<tag>/counters_*.csv        (copied counter rows of our kernels)
  profiles/<tag>/summary.json          per-kernel average duration and HBM
                                       bytes per launch (FETCH_SIZE x 2 on
                                       gfx950 + WRITE_SIZE, both in KiB)
and, if a workload key is given, that key's entry of bench_pmc.json at the
repository root for bench.py (outside profiles/, which does not travel to
the GPU box).  Keys name one rank's launch (its shard of the workload), so
an N-rank bench line reads the entry of an N = 1 run of the same shard.
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    base = name.split("(")[0].replace("void ", "")
    return base.strip()


def main(src: str, dst: str, key: str | None = None):
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace_run_kernel_stats.csv")
    kern = {}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            if "eks::" in r["Name"]:
                kern[short(r["Name"])] = dict(calls=int(r["Calls"]),
                                              avg_ms=float(r["AverageNs"]) / 1e6,
                                              total_ms=float(r["TotalDurationNs"]) / 1e6)
    traffic = defaultdict(dict)
    for kind, counter, factor in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
        path = os.path.join(src, f"pmc_{kind}_run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        shutil.copy(path, os.path.join(dst, f"counters_{kind}.csv"))
        acc = defaultdict(list)
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter and "eks::" in r["Kernel_Name"]:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            traffic[k][kind + "_bytes"] = factor * 1024.0 * sum(v) / len(v)
    summary = {"kernels": {}}
    tot_bytes = 0.0
    tot_ms = 0.0
    for k in sorted(set(kern) | set(traffic)):
        d = dict(kern.get(k, {}))
        d.update(traffic.get(k, {}))
        b = d.get("fetch_bytes", 0.0) + d.get("write_bytes", 0.0)
        d["hbm_bytes"] = b
        if "avg_ms" in d and d["avg_ms"] > 0:
            d["hbm_GBps"] = b / (d["avg_ms"] * 1e-3) / 1e9
        summary["kernels"][k] = d
        # the eks_smooth pipeline on member predictions (not the fit, not the
        # hand-off variant of K1 the bench's end-to-end loop runs)
        if ("k_c" in k or "k3_" in k or "k_model" in k or "k_smooth_seq" in k) and "YevIn" not in k:
            tot_bytes += b
            tot_ms += d.get("avg_ms", 0.0)
    summary["per_call"] = {"hbm_bytes": tot_bytes, "kernel_ms": tot_ms,
                           "hbm_GBps": tot_bytes / (tot_ms * 1e-3) / 1e9 if tot_ms else None}
    summary["notes"] = ("FETCH_SIZE doubled: on gfx950 it reports half the bytes of coalesced "
                        "streaming reads (MI355X_MICROARCH.md §HBM); checked here against each "
                        "kernel's designed byte count.")
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    if key:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        path = os.path.join(root, "bench_pmc.json")
        try:
            allpm = json.load(open(path))
        except Exception:
            allpm = {}
        entries = allpm.get("entries") or {}
        entries[key] = {"hbm_bytes_per_launch": tot_bytes, "kernel_ms": tot_ms,
                        "source": os.path.join(dst, "summary.json"),
                        "kernels": summary["kernels"]}
        json.dump({"entries": entries}, open(path, "w"), indent=1)
    print(json.dumps(summary["per_call"]))
    for k, d in summary["kernels"].items():
        print(f"  {k:40s} {d.get('avg_ms', 0):8.3f} ms  {d['hbm_bytes'] / 1e9:7.3f} GB  "
              f"{d.get('hbm_GBps', 0):8.1f} GB/s")


if __name__ == "__main__":
    main(*sys.argv[1:])
