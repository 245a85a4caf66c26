"""The device-group host logic under ThreadSanitizer (VERDICT
r4 weak 11).  `csrc/group.h` — the ThreadReducer of shards that share a GPU,
the abort protocol of a device group's non-blocking RCCL communicators
(GroupAbort) and the shard-thread driver (run_shard_threads) — is the code
libtritd's device-set route runs (api.cpp: run_threaded); here it is built
into tests/group_harness.cpp with the GPU and RCCL replaced by host models,
with -fsanitize=thread, and must run clean: sums in shard order, a shard
that throws releases every other shard, no communicator is used after the
abort frees it, no hang."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG, ROOT

HARNESS = os.path.join(ROOT, "tests", "group_harness.cpp")
CSRC = os.path.join(PKG, "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_group_logic_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "group_harness")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", f"-fsanitize={san}",
           "-fno-sanitize-recover=all", "-I", CSRC, HARNESS, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "group harness ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr


def test_library_uses_the_harnessed_header():
    """api.cpp drives device groups through group.h (not a private copy)."""
    src = open(os.path.join(CSRC, "api.cpp")).read()
    assert '#include "group.h"' in src
    assert "struct ThreadReducer" not in src
    assert "run_shard_threads(" in src and "GroupAbort" in src
