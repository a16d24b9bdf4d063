"""The in-launch hand-off protocol, checked on the machine code that ships.

The chained passes (algo 3's k3_fwd / k3_bwd, algo 2's chained scans
k_c2_fscan_g / k_c4_bscan_g) hand values between workgroups of one launch in
the form `eks_amd/csrc/handoff.hpp` documents and `MI355X_MICROARCH.md`
lists as valid on gfx950: payloads stored write-through (`sc1`), the
publishing wave drained (`s_waitcnt vmcnt(0)`), then one 32-bit flag store
(`sc1`); consumers poll flags and read payloads with `sc1` loads.  That form
is a property of the compiled code, not of the source: a toolchain that
dropped a cache bit or moved a store past the drain would still pass every
test that does not happen to race.  These tests read the disassembly of
`eks_amd/lib/libeks_hip.so` (CPU only, no GPU) and fail on any such change.

Also checked over every device function: the code object targets gfx950
only, and no function writes through the scalar data cache (every store and
atomic is a vector-memory or LDS instruction).
"""
import os
import re
import tempfile

import pytest

import isa_listing as il

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "eks_amd", "lib",
                   "libeks_hip.so")
HANDOFF_KERNELS = re.compile(r"eks::(k3_fwd|k3_bwd|k_c2_fscan_g|k_c4_bscan_g)<")

pytestmark = pytest.mark.skipif(not (os.path.exists(LIB) and il.tools_present()),
                                reason="libeks_hip.so not built or ROCm LLVM tools absent")


@pytest.fixture(scope="module")
def listing():
    with tempfile.TemporaryDirectory() as d:
        funcs, targets = il.all_functions(LIB, d)
    return funcs, targets, il.demangle(list(funcs))


def _handoff_functions(listing):
    funcs, _, dm = listing
    out = {}
    for name, body in funcs.items():
        m = HANDOFF_KERNELS.search(dm[name])
        if m:
            out.setdefault(m.group(1), []).append((dm[name], body))
    return out


def _has_sc1(line):
    return "sc1" in il.operands(line)


_VMEM_WRITE = re.compile(r"(global|buffer|flat|scratch)_(store|atomic)")


def test_code_objects_are_gfx950_only(listing):
    _, targets, _ = listing
    assert targets
    for t in targets:
        dev = [x for x in t if not x.startswith("host-")]
        assert dev == [il.TARGET], t


def test_every_chained_kernel_is_present(listing):
    found = _handoff_functions(listing)
    assert set(found) == {"k3_fwd", "k3_bwd", "k_c2_fscan_g", "k_c4_bscan_g"}
    # config 4's instantiations (r = 2, n = 2, 5 float32 members)
    assert any(n.startswith("void eks::k3_fwd<2, 2, 5, float") for n, _ in found["k3_fwd"])
    assert any(n.startswith("void eks::k3_bwd<2, 2, 5, float") for n, _ in found["k3_bwd"])


def test_flag_stores_follow_a_drain(listing):
    """Every 32-bit flag store is `sc1`, and walking back from it the wave
    meets `s_waitcnt vmcnt(0)` before any other vector-memory write: the
    payload stores that precede it in program order have completed."""
    for kind, fns in _handoff_functions(listing).items():
        for name, body in fns:
            flags = [i for i, l in enumerate(body)
                     if il.mnemonic(l) == "global_store_dword" and _has_sc1(l)]
            assert flags, f"{name}: no flag store"
            for i in flags:
                j = i - 1
                while j >= 0:
                    op = il.mnemonic(body[j])
                    if op == "s_waitcnt" and "vmcnt(0)" in body[j]:
                        break
                    assert not _VMEM_WRITE.match(op), \
                        f"{name}: '{body[j]}' not drained before flag store '{body[i]}'"
                    j -= 1
                assert j >= 0, f"{name}: flag store '{body[i]}' without a drain"
            plain32 = [l for l in body if il.mnemonic(l) == "global_store_dword" and not _has_sc1(l)]
            assert not plain32, f"{name}: 32-bit stores without sc1: {plain32[:3]}"


def test_payloads_write_through_and_polls_bypass(listing):
    for kind, fns in _handoff_functions(listing).items():
        for name, body in fns:
            ops = [(il.mnemonic(l), _has_sc1(l)) for l in body]
            assert ("global_store_dwordx2", True) in ops, f"{name}: no write-through payload store"
            assert ("global_load_dword", True) in ops, f"{name}: no sc1 flag poll"
            assert ("global_load_dwordx2", True) in ops, f"{name}: no sc1 payload load"


def test_no_scalar_cache_writes(listing):
    funcs, _, dm = listing
    assert len(funcs) > 100
    bad = []
    for name, body in funcs.items():
        for l in body:
            op = il.mnemonic(l)
            if op.startswith("s_") and ("store" in op or "atomic" in op or op.endswith("_wb")):
                bad.append((dm[name], l))
    assert not bad, bad[:5]
