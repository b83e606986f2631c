"""dcf_amd — MI355X-native batch evaluator for the `dcf` crate's distributed
comparison function (xymeng16/dcf v0.2.2).

The compute lives in ``libdcf_hip.so`` (HIP kernels for gfx950 behind the C ABI
of include/dcf_hip.h).  This package is the host-side mirror of the crate's
`Dcf` / `Prg` interface; it has no CPU compute path.
"""
from ._lib import DcfError, LIB_PATH, load  # noqa: F401
from .dcf import (  # noqa: F401
    Aes128MatyasMeyerOseasPrg,
    Aes256HirosePrg,
    BoundState,
    CmpFn,
    Cw,
    DcfImpl,
    MultiGpuDcf,
    Share,
    cwb_bytes,
    cwb_np1_offset,
    cwb_to_share,
    point_slice,
    share_to_cwb,
)

__all__ = [
    "Aes128MatyasMeyerOseasPrg", "Aes256HirosePrg", "BoundState", "CmpFn", "Cw", "DcfImpl", "MultiGpuDcf", "Share", "point_slice", "DcfError",
    "cwb_bytes", "cwb_np1_offset", "cwb_to_share", "share_to_cwb", "load", "LIB_PATH",
]
