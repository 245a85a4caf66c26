"""No wide store in the shipped gfx950 code has its data registers rewritten
by a VALU / MFMA instruction within two issued instructions (VERDICT r4 next
1).  On MI355X such a rewrite replaces the stored data of lanes
12-15 of each 16, and LLVM pads it only for stores it considers hazardous —
not for buffer stores with an SGPR soffset, the form K5 streams through
(tools/scan_store_war.py docstring, DESIGN.md §4.2, the probe in
profiles/round5/store_hazard_probe.txt).  The keeps in k_admm.hip are what
hold the compiler off; this test is what makes them mechanical: it scans
every code object of libtritd.so, and checks that a K5 compiled without the
keeps IS caught."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import scan_store_war as sw  # noqa: E402

LIB = os.path.join(PKG, "tritd", "libtritd.so")
CSRC = os.path.join(PKG, "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(f"{sw.LLVM}/llvm-objdump"),
                                reason="llvm-objdump not installed")


def _fmt(hits):
    return "\n".join(f"{f}: 0x{a:x} {st} <- +{d} {w}" for f, hs in hits.items()
                     for a, st, d, w in hs)


def test_shipped_library_has_no_wide_store_data_rewrite():
    assert os.path.exists(LIB), "build libtritd.so first (__graft_entry__.build())"
    hits = sw.scan_object(LIB, sw.WINDOW, sync_only=True)
    assert not hits, "wide-store data rewritten too early:\n" + _fmt(hits)


def test_scan_sees_every_kernel_file():
    """The scan covers all eight kernel files' code objects (one offload bundle
    each), K5 included."""
    blobs = sw.code_objects(LIB)
    assert len(blobs) >= 8
    funs = set()
    for b in blobs:
        funs |= set(sw.parse(sw.disassemble(b)))
    for k in ("k5_fused", "k5_f32s", "k_m3_cp", "k_tp", "k_transpose", "k_soft_threshold", "k_als_fit"):
        assert any(k in f for f in funs), k


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_k5_without_the_keeps_is_caught(tmp_path):
    """The round-4 failing form: K5 built with TRITD_STORE_KEEP=0 has the
    compiler write a data pair right behind a buffer_store_dwordx4 (it
    reproduces the corruption on the GPU: profiles/round5/
    nokeep_determinism.txt).  The scan must flag it in the dense-E K5."""
    obj = str(tmp_path / "k_admm_nokeep.o")
    cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I" + os.path.join(ROOT, "include"),
           "-I" + CSRC, "--offload-arch=gfx950", "-DTRITD_STORE_KEEP=0", "-c",
           os.path.join(CSRC, "k_admm.hip"), "-o", obj]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    hits = sw.scan_object(obj, sw.WINDOW, sync_only=True)
    dense_e = {f: h for f, h in hits.items() if "k5_fused" in f and "Lb0ELb1E" in f}
    assert dense_e, "the scan missed the keep-less dense-E K5:\n" + _fmt(hits)
    assert any(d == 1 for hs in dense_e.values() for _, _, d, _ in hs)
