"""Debug: does a GPU test file leave a stale HIP error / break torch's later
initialisation?  Runs the file in-process, then reports hipGetLastError() and
tries torch.cuda."""
import ctypes as C
import sys

import pytest

hip = C.CDLL("libamdhip64.so")
hip.hipGetLastError.restype = C.c_int
for f in sys.argv[1:]:
    for t in pytest.main([f, "-m", "gpu", "-q", "-p", "no:cacheprovider", "--co", "-q"]) and [] or []:
        pass
    rc = pytest.main([f, "-m", "gpu", "-q", "-x", "-p", "no:cacheprovider"])
    print("==", f, "rc", rc, "hipGetLastError after:", hip.hipGetLastError(), flush=True)
import torch  # noqa: E402
try:
    x = torch.zeros(4, device="cuda")
    print("torch ok", x.sum().item(), flush=True)
except Exception as e:  # noqa: BLE001
    print("torch failed:", e, flush=True)
