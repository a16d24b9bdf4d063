"""Disassembly of the shipped device code (test infrastructure, CPU only).

Extracts the gfx950 code objects that ``eks_amd/lib/libeks_hip.so`` carries
in its ``.hip_fatbin`` section (one offload bundle per translation unit,
compressed or not), disassembles them with the ROCm LLVM tools and splits the
listing into functions, so that tests can check properties of the machine
code that ships -- not of a rebuild.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
from concurrent.futures import ThreadPoolExecutor

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
_CCOB = b"CCOB"                           # compressed bundle magic
_PLAIN = b"__CLANG_OFFLOAD_BUNDLE__"      # uncompressed bundle magic


def tools_present() -> bool:
    return all(os.path.exists(os.path.join(LLVM, t))
               for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump"))


def _run(*args: str) -> str:
    return subprocess.run(args, check=True, capture_output=True, text=True).stdout


def _bundles(blob: bytes) -> list[bytes]:
    """Split a .hip_fatbin section into its offload bundles (4 KB aligned)."""
    starts = sorted({m.start() for m in re.finditer(re.escape(_CCOB), blob)}
                    | {m.start() for m in re.finditer(re.escape(_PLAIN), blob)})
    out = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(blob)
        b = blob[s:e]
        if b.startswith(_CCOB):
            ver = struct.unpack_from("<H", b, 4)[0]
            # v2: 32-bit total size at 8; v3: 64-bit total size at 8
            tot = struct.unpack_from("<I" if ver == 2 else "<Q", b, 8)[0]
            b = b[:tot]
        out.append(b)
    return out


def code_objects(lib: str, workdir: str) -> list[tuple[str, list[str]]]:
    """[(path of the gfx950 code object, targets listed in its bundle)]"""
    fb = os.path.join(workdir, "fatbin.bin")
    _run(os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", lib,
         os.path.join(workdir, "stripped.so"))
    res = []
    for i, b in enumerate(_bundles(open(fb, "rb").read())):
        bp = os.path.join(workdir, f"bundle{i}.bin")
        open(bp, "wb").write(b)
        bundler = os.path.join(LLVM, "clang-offload-bundler")
        targets = _run(bundler, "--list", "--type=o", f"--input={bp}").split()
        co = os.path.join(workdir, f"co{i}.o")
        _run(bundler, "--unbundle", "--type=o", f"--input={bp}", f"--targets={TARGET}",
             f"--output={co}")
        res.append((co, targets))
    return res


_FUNC = re.compile(r"^[0-9a-f]+ <(_Z[^>]*|[A-Za-z_][^>]*)>:$")
_LABEL = re.compile(r"^[0-9a-f]+ <L\d+>:$")


def functions(listing: str) -> dict[str, list[str]]:
    """{mangled function name: [instruction or label lines]} of one listing"""
    funcs: dict[str, list[str]] = {}
    cur = None
    for raw in listing.splitlines():
        line = raw.split("//")[0].strip()
        if not line:
            continue
        if _LABEL.match(line):
            if cur is not None:
                funcs[cur].append("<label>")
            continue
        m = _FUNC.match(line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None and not line.startswith("Disassembly") and ":" not in line.split()[0]:
            funcs[cur].append(line)
    return funcs


def disassemble(co: str) -> dict[str, list[str]]:
    return functions(_run(os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950",
                          "--no-show-raw-insn", "--symbolize-operands", co))


def all_functions(lib: str, workdir: str) -> tuple[dict[str, list[str]], list[list[str]]]:
    """Every device function of the library (merged over its code objects)
    and the target list of every bundle."""
    cos = code_objects(lib, workdir)
    with ThreadPoolExecutor(max_workers=min(8, len(cos) or 1)) as ex:
        parts = list(ex.map(disassemble, [c for c, _ in cos]))
    funcs: dict[str, list[str]] = {}
    for p in parts:
        funcs.update(p)
    return funcs, [t for _, t in cos]


def demangle(names: list[str]) -> dict[str, str]:
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    return dict(zip(names, out))


def mnemonic(line: str) -> str:
    return line.split()[0]


def operands(line: str) -> list[str]:
    return line.replace(",", " ").split()[1:]
