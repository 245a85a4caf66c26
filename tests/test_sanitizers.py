"""SURVEY.md §5 aux: ASan/UBSan builds of the host-side code that is not HIP —
the C restatement of the reference (oracle/tritd_ref.c) and the MEX gateway
over the mock mx runtime — run as standalone executables (no interpreter, so
no preloading: the sanitizer runtime is linked in).  GPU code is never built
with sanitizers (the pool refuses GPU ASan)."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG, ROOT

SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2")


def _run(exe):
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "ERROR: AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "LeakSanitizer" not in p.stderr, p.stderr[-4000:]
    return p.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_c_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "ref_driver")
    subprocess.run(["gcc", "-O1", "-g", "-std=c11", "-fopenmp", "-ffp-contract=off", *SAN,
                    os.path.join(ROOT, "tests", "sanitize", "ref_driver.c"),
                    os.path.join(ROOT, "oracle", "tritd_ref.c"), "-o", exe, "-lm"], check=True)
    assert "ok" in _run(exe)


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_mex_gateway_under_asan_ubsan(tmp_path):
    libdir = os.path.join(PKG, "tritd")
    if not os.path.exists(os.path.join(libdir, "libtritd.so")):
        pytest.skip("libtritd.so not built")
    exe = str(tmp_path / "mex_driver")
    mock = os.path.join(ROOT, "tests", "mock_mex")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", *SAN, "-I" + mock, "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "sanitize", "mex_driver.cpp"),
                    os.path.join(PKG, "matlab", "tritd_mex.cpp"), os.path.join(mock, "mock_mex.cpp"),
                    "-L" + libdir, "-ltritd", "-Wl,-rpath," + libdir, "-o", exe], check=True)
    assert "mex_driver: ok" in _run(exe)
