"""Static ISA census of device kernels in a hipcc ``-S`` listing.

Usage: python tools/isa_count.py file.s [kernel-regex]

For each kernel symbol matching the regex prints VGPR/AGPR/SGPR counts,
LDS bytes, occupancy (waves/SIMD) and instruction counts per class
(v_*_f64, other VALU, SALU, global/buffer memory, LDS, branches).
Used for the ISA counts committed under profiles/.
"""
import collections
import re
import sys


def census(path, rx):
    kern = None
    counts = {}
    meta = {}
    pat = re.compile(rx)
    for line in open(path):
        s = line.split(";")[0].strip() if not line.lstrip().startswith(";") else line.strip()
        if s.endswith(":") and not s.startswith(".") and not s.startswith(";"):
            name = s[:-1]
            if pat.search(name) and not name.startswith("$") and "." not in name[:2]:
                kern = name
                counts[kern] = collections.Counter()
            continue
        if kern is None:
            continue
        if s.startswith(".Lfunc_end"):
            kern = None
            continue
        if s.startswith(";") and kern:
            m = re.match(r";\s*(NumVgprs|NumAgprs|NumSgprs|ScratchSize|Occupancy|LDSByteSize|TotalNumVgprs):\s*(\d+)", s)
            if m:
                meta.setdefault(kern, {})[m.group(1)] = int(m.group(2))
            continue
        if not s or s.startswith(".") or s.startswith(";"):
            continue
        op = s.split()[0]
        c = counts[kern]
        c["total"] += 1
        if op.startswith("v_"):
            c["valu_f64" if "f64" in op else "valu"] += 1
        elif op.startswith("s_"):
            c["branch" if "branch" in op or "cbranch" in op else "salu"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
    # metadata comments follow .Lfunc_end, gather them in a second pass
    cur = None
    for line in open(path):
        s = line.strip()
        lab = line.split(";")[0].strip()
        if lab.endswith(":") and not lab.startswith("."):
            cur = lab[:-1] if lab[:-1] in counts else None
        if cur and s.startswith(";"):
            m = re.match(r";\s*(NumVgprs|NumAgprs|NumSgprs|ScratchSize|Occupancy|LDSByteSize|TotalNumVgprs):\s*(\d+)", s)
            if m:
                meta.setdefault(cur, {})[m.group(1)] = int(m.group(2))
    return counts, meta


def demangle(name):
    try:
        import subprocess
        return subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt", name], capture_output=True,
                              text=True).stdout.strip()
    except OSError:
        return name


def main():
    path = sys.argv[1]
    rx = sys.argv[2] if len(sys.argv) > 2 else "."
    counts, meta = census(path, rx)
    for k in counts:
        c, m = counts[k], meta.get(k, {})
        print(demangle(k)[:150])
        print("  vgpr %s agpr %s sgpr %s lds %s scratch %s occ %s" % (
            m.get("NumVgprs"), m.get("NumAgprs"), m.get("NumSgprs"), m.get("LDSByteSize"),
            m.get("ScratchSize"), m.get("Occupancy")))
        print("  " + " ".join(f"{key} {c[key]}" for key in
                              ("total", "valu_f64", "valu", "salu", "vmem", "lds", "branch")))


if __name__ == "__main__":
    main()
