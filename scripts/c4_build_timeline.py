"""C4 wide shared-prefix build timeline from in-kernel stamps (diagnostic build,
-DDCF_CLOCK_STAMPS): where k_wpfx_build's time goes between the LDS table fill, the root path
(wave 0, levels 0 .. S-1), the workgroup levels S .. D-4 and the last three levels, relative to
the first workgroup's stamp after its fill (s_memrealtime, 100 MHz).

  DCF_HIP_LIB=dcf_amd/libdcf_hip_clk.so python scripts/c4_build_timeline.py > c4_build.json
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dcf_amd  # noqa: E402
from dcf_amd import _lib  # noqa: E402

GROUPS = 4096


def slot(lib, s):
    buf = (ctypes.c_uint64 * (GROUPS * 4))()
    assert lib.dcf_debug_clock_stamps(0, s, buf, GROUPS * 4) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(GROUPS, 4).astype(np.int64)


def main():
    lib = _lib.load()
    lib.dcf_debug_clock_stamps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    lib.dcf_debug_clock_reset.argtypes = [ctypes.c_int]
    rng = np.random.default_rng(0xDCF0004)
    lam, nb = 16384, 16
    prg = dcf_amd.Aes256HirosePrg([rng.bytes(32) for _ in range(18)], lam)
    d = dcf_amd.DcfImpl(nb, lam, prg)
    k = d.gen(dcf_amd.CmpFn(rng.bytes(nb), rng.bytes(lam)), [rng.bytes(lam), rng.bytes(lam)],
              dcf_amd.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, nb, lam), np.uint8).copy()).cuda()
    s0 = torch.from_numpy(np.frombuffer(k.s0s[0], np.uint8).copy()).cuda()
    m = int(os.environ.get("C4_POINTS", str(1 << 22)))
    xs = torch.randint(0, 256, (m, nb), dtype=torch.uint8, device="cuda")
    ys = torch.empty((m, lam), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    lib.dcf_debug_clock_reset(0)
    torch.cuda.synchronize()
    d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    a, b, head = slot(lib, 6), slot(lib, 7), slot(lib, 5)
    live = a[:, 1] > 0
    ref = a[live, 1].min()

    def dist(x):
        x = (x - ref) / 1e5
        return {"first": float(x.min()), "median": float(np.median(x)), "last": float(x.max()), "n": int(len(x))}

    out = {"workgroups": int(live.sum()), "prefix_levels": prg.eval_prefix_levels(nb, 1, m),
           "after_fill": dist(a[live, 1]), "root_path_done": dist(a[live, 3]),
           "last3_levels_start": dist(b[live, 1]), "build_done": dist(b[live, 3]),
           "head_entry": dist(head[head[:, 1] > 0, 1]),
           "note": "ms relative to the first build workgroup's stamp after its LDS table fill (s_memrealtime)"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
