"""Engine clock during C4 (and C3 for reference) by two methods independent of the
GRBM_GUI_ACTIVE / kernel-time quotient (VERDICT r02 "What's weak" 3):

1. in-kernel stamps (MI355X_MICROARCH.md "DVFS give-back" item 6): a diagnostic build
   (scripts/build_variant.sh clk -DDCF_CLOCK_STAMPS) stamps s_memtime (shader clock) and
   s_memrealtime (100 MHz) per workgroup at the start and end of k_eval_wide_tail2,
   k_eval_wide_head_stream and k_eval16_stream; clock = d(memtime) / d(realtime) x 100 MHz;
2. amd-smi sampling from a second process while the loop runs (if amd-smi works on the box).

  DCF_HIP_LIB=dcf_amd/libdcf_hip_clk.so python scripts/clock_probe.py > clock.json
"""
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dcf_amd  # noqa: E402
from dcf_amd import _lib  # noqa: E402

GROUPS = 4096
SLOTS = {0: "k_eval_wide_tail2", 1: "k_eval_wide_head_stream", 2: "k_eval16_stream"}


def stamps(lib, slot):
    buf = (ctypes_u64 * (GROUPS * 4))()
    rc = lib.dcf_debug_clock_stamps(0, slot, buf, GROUPS * 4)
    assert rc == 0, rc
    a = np.frombuffer(buf, dtype=np.uint64).reshape(GROUPS, 4).astype(np.int64)
    live = (a[:, 1] > 0) & (a[:, 3] > a[:, 1])
    a = a[live]
    if not len(a):
        return None
    dt, dr = a[:, 2] - a[:, 0], a[:, 3] - a[:, 1]
    ghz = dt / dr * 0.1  # realtime ticks at 100 MHz
    span = (a[:, 3].max() - a[:, 1].min()) / 1e5  # ms from the first start to the last end
    return {"workgroups": int(len(a)), "clock_ghz_median": float(np.median(ghz)), "clock_ghz_min": float(ghz.min()),
            "clock_ghz_max": float(ghz.max()), "clock_ghz_cycle_weighted": float(dt.sum() / dr.sum() * 0.1),
            "wg_ms_median": float(np.median(dr) / 1e5), "launch_span_ms": float(span)}


def summ(sample):
    """socket power (W) and the mean gfx clock (MHz) over the XCDs of one amd-smi sample."""
    try:
        g = sample["out"]["gpu_data"][0] if isinstance(sample["out"], dict) else sample["out"][0]
        clks = [v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_") and isinstance(v, dict)
                and isinstance(v.get("clk"), dict) and isinstance(v["clk"].get("value"), (int, float))]
        return {"t": sample["t"], "socket_power_w": g["power"]["socket_power"]["value"],
                "gfx_mhz_mean": sum(clks) / len(clks) if clks else None}
    except Exception as e:  # noqa: BLE001
        return {"t": sample["t"], "parse_error": repr(e)}


class Smi(threading.Thread):
    """amd-smi metric sampling in a subprocess loop (best effort)."""

    def __init__(self):
        super().__init__(daemon=True)
        self.samples, self.err, self.stop = [], None, False

    def run(self):
        while not self.stop:
            try:
                r = subprocess.run(["amd-smi", "metric", "-g", "0", "-c", "-p", "--json"], capture_output=True,
                                   text=True, timeout=20)
                if r.returncode != 0:
                    self.err = (r.stderr or r.stdout)[-400:]
                    return
                self.samples.append({"t": time.time(), "out": json.loads(r.stdout)})
            except Exception as e:  # noqa: BLE001
                self.err = repr(e)
                return
            time.sleep(0.05)


def c4_loop(steps):
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
    for _ in range(3):
        d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    del ys
    return ms


def c3_loop(steps):
    rng = np.random.default_rng(0xDCF0001)
    keys = [rng.bytes(32) for _ in range(2)]
    prg = dcf_amd.Aes256HirosePrg(keys, 16)
    d = dcf_amd.DcfImpl(16, 16, prg)
    k = d.gen(dcf_amd.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf_amd.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, 16, 16), np.uint8).copy()).cuda()
    s0 = torch.from_numpy(np.frombuffer(k.s0s[0], np.uint8).copy()).cuda()
    xs = torch.randint(0, 256, (1 << 28, 16), dtype=torch.uint8, device="cuda")
    ys = torch.empty((1 << 28, 16), dtype=torch.uint8, device="cuda")
    d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


ctypes_u64 = None


def main():
    global ctypes_u64
    import ctypes
    ctypes_u64 = ctypes.c_uint64
    lib = _lib.load()
    lib.dcf_debug_clock_stamps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    out = {"lib": _lib.LIB_PATH}
    smi = Smi()
    smi.start()
    out["c4_ms_per_step"] = c4_loop(int(os.environ.get("C4_STEPS", "60")))
    smi.stop = True
    smi.join()
    out["c4"] = {SLOTS[s]: stamps(lib, s) for s in (0, 1)}
    out["amd_smi_c4"] = {"samples": [summ(x) for x in smi.samples], "error": smi.err}
    smi = Smi()
    smi.start()
    out["c3_ms_per_step"] = c3_loop(int(os.environ.get("C3_STEPS", "6")))
    smi.stop = True
    smi.join()
    out["c3"] = {SLOTS[2]: stamps(lib, 2)}
    out["amd_smi_c3"] = {"samples": [summ(x) for x in smi.samples], "error": smi.err}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
