"""Where a single-point dcf_eval's time goes: the in-kernel duration and engine clock of
k_eval16_oct (clock stamps of a -DDCF_CLOCK_STAMPS build, slot 3) beside the per-call time.
  DCF_HIP_LIB=dcf_amd/libdcf_hip_clk.so python scripts/lat_probe.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dcf_amd  # noqa: E402
from dcf_amd import _lib  # noqa: E402
from dcf_amd.dcf import _ptr  # noqa: E402

rng = np.random.default_rng(5)
keys = [rng.bytes(32) for _ in range(2)]
prg = dcf_amd.Aes256HirosePrg(keys, 16)
d = dcf_amd.DcfImpl(16, 16, prg)
k = d.gen(dcf_amd.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf_amd.BoundState.LtBeta)
lib = _lib.load()
lib.dcf_debug_clock_stamps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
cwb = np.frombuffer(dcf_amd.share_to_cwb(k, 16, 16), np.uint8).copy()
s0 = bytes(k.s0s[0])
xb = np.frombuffer(rng.bytes(16), np.uint8).copy()
yb = np.zeros(16, np.uint8)
out = {}
for rep in range(3):
    n = 300
    t0 = time.perf_counter()
    for _ in range(n):
        assert lib.dcf_eval(prg.handle, 16, 0, _ptr(cwb), cwb.size, _ptr(s0), _ptr(xb), 1, _ptr(yb), 16) == 0
    us = (time.perf_counter() - t0) / n * 1e6
    buf = (ctypes.c_uint64 * (4096 * 4))()
    assert lib.dcf_debug_clock_stamps(0, 3, buf, 4096 * 4) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4).astype(np.int64)[0]
    out[rep] = {"us_per_call": us, "kernel_walk_us": (a[3] - a[1]) / 100.0,
                "clock_ghz": (a[2] - a[0]) / (a[3] - a[1]) * 0.1 if a[3] > a[1] else None}
print(json.dumps(out), flush=True)
