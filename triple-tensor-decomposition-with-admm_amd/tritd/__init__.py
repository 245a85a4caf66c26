"""tritd — MI355X-native TriTD-ADMM (drop-in for triple_decomp_ADMM).

Import with the package directory on sys.path:

    sys.path.insert(0, "<repo>/triple-tensor-decomposition-with-admm_amd")
    import tritd
    A, B, C, O, errHist = tritd.triple_decomp_ADMM(D, r, opts)
"""
from ._lib import LIB_PATH, PinvToleranceWarning, TritdError, device_count, set_devices, set_printer, shutdown  # noqa: F401
from .api import (  # noqa: F401
    AlsSession,
    Comm,
    Session,
    buildF,
    buildG,
    buildH,
    evaluate,
    initial_factors,
    make_opts,
    quality_ybz,
    soft_threshold,
    triple_decomp_ADMM,
    triple_decomp_ADMM_outlier,
    triple_decomp_ncvx,
    triple_decomp_ALS,
    triple_product,
    unfold,
)

__version__ = "0.1.0"
