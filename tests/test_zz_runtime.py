"""Runs last in the GPU suite (file order): the suite's own process used
libtritd on /opt/rocm's HIP runtime — the runtime the MEX drop-in binds —
and never loaded a second one (torch-interop checks run in child processes,
tests/test_gpu_devprod.py)."""
import sys

import pytest


@pytest.mark.gpu
def test_suite_process_ran_on_the_system_hip_runtime():
    if "tritd._lib" not in sys.modules:
        pytest.skip("tritd not loaded in this process")
    from tritd._lib import HIP_RUNTIME, hip_runtimes
    assert "torch" not in sys.modules, "a GPU test imported torch into the suite's process"
    assert hip_runtimes() == [HIP_RUNTIME], hip_runtimes()
    assert HIP_RUNTIME.startswith("/opt/rocm"), HIP_RUNTIME
