"""C4 step timeline from in-kernel stamps (diagnostic build, -DDCF_CLOCK_STAMPS): where the
~34 ms of one LAMBDA = 16384 eval of 2^22 points go.  Every workgroup of the last launch of
k_eval_wide_head_stream and k_eval_wide_tail2 stamps s_memrealtime (100 MHz, one clock for
the whole chip) at entry, after its LDS table build, and at the end of its main loop; the
timeline is relative to the first head workgroup's entry.

  DCF_HIP_LIB=dcf_amd/libdcf_hip_clk.so python scripts/c4_timeline.py > c4_timeline.json
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
    a = np.frombuffer(buf, dtype=np.uint64).reshape(GROUPS, 4).astype(np.int64)
    return a


def main():
    lib = _lib.load()
    lib.dcf_debug_clock_stamps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    lib.dcf_debug_clock_reset.argtypes = [ctypes.c_int]
    rng = np.random.default_rng(0xDCF0001)
    keys = [rng.bytes(32) for _ in range(2048)]
    prg = dcf_amd.Aes256HirosePrg(keys, 16384)
    d = dcf_amd.DcfImpl(16, 16384, prg)
    k = d.gen(dcf_amd.CmpFn(rng.bytes(16), rng.bytes(16384)), [rng.bytes(16384), rng.bytes(16384)],
              dcf_amd.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, 16, 16384), np.uint8).copy()).cuda()
    s0 = torch.from_numpy(np.frombuffer(k.s0s[0], np.uint8).copy()).cuda()
    xs = torch.randint(0, 256, (1 << 22, 16), dtype=torch.uint8, device="cuda")
    ys = torch.empty((1 << 22, 16384), dtype=torch.uint8, device="cuda")
    steps = int(os.environ.get("C4_STEPS", "20"))
    for _ in range(3):
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
    tail_loop, head_walk = slot(lib, 0), slot(lib, 1)
    tail_in, head_in = slot(lib, 4), slot(lib, 5)

    def live(a, col):
        return a[a[:, col] > 0, col]

    hi, ti = live(head_in, 1), live(tail_in, 1)
    hw0, hw1 = live(head_walk, 1), live(head_walk, 3)
    tl0, tl1 = live(tail_loop, 1), live(tail_loop, 3)
    ref = hi.min()

    def ms_(x):
        return float((x - ref) / 1e5)

    def dist(x):
        return {"first": ms_(x.min()), "median": ms_(np.median(x)), "last": ms_(x.max()), "n": int(len(x))}

    out = {"c4_ms_per_step": ms, "one_eval_event_ms": one_ms,
           "head_entry": dist(hi), "head_walk_start": dist(hw0), "head_walk_end": dist(hw1),
           "tail_entry": dist(ti), "tail_loop_start": dist(tl0), "tail_loop_end": dist(tl1),
           "head_table_fill_ms_median": float(np.median((head_walk[:, 1] - head_in[:, 1])[(head_in[:, 1] > 0) & (head_walk[:, 1] > 0)]) / 1e5),
           "tail_table_build_ms_median": float(np.median((tail_loop[:, 1] - tail_in[:, 1])[(tail_in[:, 1] > 0) & (tail_loop[:, 1] > 0)]) / 1e5),
           "note": "s_memrealtime stamps (100 MHz) of the last eval; ms relative to the first head workgroup's entry"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
