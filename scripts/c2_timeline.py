"""C2 step timeline from in-kernel stamps (diagnostic build, -DDCF_CLOCK_STAMPS): where one
N = 4, LAMBDA = 16 eval of 2^24 points goes between the shared-prefix table build
(k_prefix_build16: table fill, root path, breadth-first levels, depth-first tail) and the walk
(k_eval16_stream).  Lane 0 of every workgroup stamps s_memrealtime (100 MHz, one clock for the
chip); the timeline is relative to the first build workgroup's entry.

  DCF_HIP_LIB=dcf_amd/libdcf_hip_clk.so python scripts/c2_timeline.py > c2_timeline.json
"""
import ctypes
import json
import os
import sys
import time

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
    rng = np.random.default_rng(0xDCF0002)
    prg = dcf_amd.Aes256HirosePrg([rng.bytes(32)], 16)
    d = dcf_amd.DcfImpl(4, 16, prg)
    k = d.gen(dcf_amd.CmpFn(rng.bytes(4), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)],
              dcf_amd.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, 4, 16), np.uint8).copy()).cuda()
    s0 = torch.from_numpy(np.frombuffer(k.s0s[0], np.uint8).copy()).cuda()
    m = int(os.environ.get("C2_POINTS", str(1 << 24)))
    xs = torch.randint(0, 256, (m, 4), dtype=torch.uint8, device="cuda")
    ys = torch.empty((m, 16), dtype=torch.uint8, device="cuda")
    steps = int(os.environ.get("C2_STEPS", "60"))
    for _ in range(5):
        d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    lib.dcf_debug_clock_reset(0)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    d.eval_device(False, cwb, s0, xs, ys)
    ev[1].record()
    torch.cuda.synchronize()
    one_ms = ev[0].elapsed_time(ev[1])
    b_fill, b_root, walk = slot(lib, 6), slot(lib, 7), slot(lib, 2)

    def live(a, col):
        return a[a[:, col] > 0, col]

    ref = live(b_fill, 1).min()

    def dist(x):
        x = (x - ref) / 1e5
        return {"first": float(x.min()), "median": float(np.median(x)), "last": float(x.max()), "n": int(len(x))}

    out = {"c2_ms_per_step": ms, "one_eval_event_ms": one_ms,
           "build_entry_after_fill": dist(live(b_fill, 1)), "build_root_path_done": dist(live(b_root, 1)),
           "build_bfs_done": dist(live(b_fill, 3)), "build_done_last_wave": dist(live(b_root, 3)),
           "walk_entry_after_fill": dist(live(walk, 1)), "walk_end_wave0": dist(live(walk, 3)),
           "note": "s_memrealtime stamps (100 MHz) of the last eval; ms relative to the first build "
                   "workgroup's stamp after its LDS table fill"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
