"""ctypes binding of the C ABI in include/dcf_hip.h (libdcf_hip.so).

There is no CPU fallback: if the HIP library is missing or cannot be loaded,
importing the compute API raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DCF_HIP_LIB: an alternative in-tree build of the same library (kernel-variant experiments).
LIB_PATH = os.environ.get("DCF_HIP_LIB") or os.path.join(_HERE, "libdcf_hip.so")

DCF_OK = 0
EVAL_AUTO, EVAL_TTABLE, EVAL_STREAM = 0, 1, 4
ERRORS = {
    -1: "DCF_ERR_ARG",
    -2: "DCF_ERR_LAMBDA",
    -3: "DCF_ERR_CIPHER_N",
    -4: "DCF_ERR_N",
    -5: "DCF_ERR_LEN",
    -6: "DCF_ERR_HIP",
    -7: "DCF_ERR_UNSUPPORTED",
    -8: "DCF_ERR_KEY",
}

# Every symbol the header declares (tests check the library exports all of them).
EXPORTS = [
    "dcf_version", "dcf_last_error", "dcf_hirose_prg_new", "dcf_mmo_prg_new", "dcf_prg_kind", "dcf_prg_free", "dcf_prg_lambda", "dcf_prg_set_eval_mode",
    "dcf_prg_last_eval_blocks", "dcf_prg_set_prefix_levels", "dcf_eval_prefix_levels",
    "dcf_eval_keys_per_launch", "dcf_cwb_bytes", "dcf_cwb_np1_offset", "dcf_gen", "dcf_eval", "dcf_prg_gen",
    "dcf_gen_batch_device", "dcf_eval_device", "dcf_eval_multikey_device", "dcf_eval_full_domain_device",
    "dcf_share_bincode_bytes", "dcf_share_to_bincode", "dcf_share_from_bincode",
    "dcf_point_slice", "dcf_eval_multi_gpu", "dcf_eval_multi_gpu_device", "dcf_prg_set_prefix_max_bytes",
    "dcf_prg_device_bytes", "dcf_prg_host_pinned_bytes", "dcf_prg_workspaces", "dcf_prg_trim", "dcf_prg_set_phase_timing",
    "dcf_prg_last_eval_phases",
]


class DcfError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


_lib = None


def load(path: str = LIB_PATH):
    """Load libdcf_hip.so (no compute happens here; safe without a GPU)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: run `python -m dcf_amd.build` (hipcc, gfx950)")
    # One HIP runtime per process: torch ships its own libamdhip64 (same soname,
    # libamdhip64.so.7).  Loading torch first makes the dynamic loader bind this
    # library to torch's runtime instead of mapping /opt/rocm's as a second one,
    # which would see no device once torch owns it.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    vp, sz, i, u8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p
    sig = {
        "dcf_version": ([], ctypes.c_char_p),
        "dcf_last_error": ([], ctypes.c_char_p),
        "dcf_hirose_prg_new": ([u8p, sz, sz, i, ctypes.POINTER(vp)], i),
        "dcf_mmo_prg_new": ([u8p, sz, sz, i, ctypes.POINTER(vp)], i),
        "dcf_prg_kind": ([vp], i),
        "dcf_prg_free": ([vp], None),
        "dcf_prg_lambda": ([vp], sz),
        "dcf_prg_set_eval_mode": ([vp, i], i),
        "dcf_prg_last_eval_blocks": ([vp, ctypes.POINTER(ctypes.c_uint64)], i),
        "dcf_prg_set_prefix_levels": ([vp, i], i),
        "dcf_eval_prefix_levels": ([vp, sz, sz, sz], i),
        "dcf_eval_keys_per_launch": ([sz, sz], sz),
        "dcf_cwb_bytes": ([sz, sz, sz], sz),
        "dcf_cwb_np1_offset": ([sz, sz, sz], sz),
        "dcf_gen": ([vp, sz, u8p, u8p, u8p, u8p, i, u8p], i),
        "dcf_eval": ([vp, sz, i, u8p, sz, u8p, u8p, sz, u8p, sz], i),
        "dcf_prg_gen": ([vp, u8p, sz, u8p], i),
        "dcf_gen_batch_device": ([vp, sz, sz, u8p, u8p, u8p, u8p, i, u8p, vp], i),
        "dcf_eval_device": ([vp, sz, i, u8p, u8p, u8p, sz, u8p, vp], i),
        "dcf_eval_multikey_device": ([vp, sz, sz, sz, i, u8p, u8p, u8p, u8p, vp], i),
        "dcf_eval_full_domain_device": ([vp, sz, i, u8p, u8p, u8p, vp], i),
        "dcf_share_bincode_bytes": ([sz, sz, sz], sz),
        "dcf_share_to_bincode": ([sz, sz, u8p, u8p, sz, u8p, sz], i),
        "dcf_share_from_bincode": ([sz, sz, u8p, sz, u8p, u8p, sz, ctypes.POINTER(sz)], i),
        "dcf_point_slice": ([sz, sz, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)], None),
        "dcf_prg_set_prefix_max_bytes": ([vp, sz], i),
        "dcf_prg_device_bytes": ([vp], sz),
        "dcf_prg_host_pinned_bytes": ([vp], sz),
        "dcf_prg_workspaces": ([vp], i),
        "dcf_prg_trim": ([vp], i),
        "dcf_prg_set_phase_timing": ([vp, i], i),
        "dcf_prg_last_eval_phases": ([vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                      ctypes.POINTER(i)], i),
        "dcf_eval_multi_gpu": ([ctypes.POINTER(vp), sz, sz, i, u8p, sz, u8p, u8p, sz, u8p, sz], i),
        "dcf_eval_multi_gpu_device": ([ctypes.POINTER(vp), sz, sz, i, u8p, sz, u8p, ctypes.POINTER(vp),
                                       ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(vp), u8p], i),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(rc: int):
    if rc != DCF_OK:
        raise DcfError(rc, load().dcf_last_error().decode(errors="replace"))
