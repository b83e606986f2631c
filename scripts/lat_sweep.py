"""Per-call time of small device-resident eval / gen batches (the latency kernels' range).

  DCF_HIP_LIB=... python scripts/lat_sweep.py > out.json

Run once per library variant (scripts/build_variant.sh: DCF_EVAL_OCT_MAX / DCF_GEN_COL_MAX)
to place the thresholds of kernels_lat.h against the pair / quad kernels.  Prints one JSON
line: {"lib": ..., "eval_us": {m: us}, "gen_us": {K: us}, "host_eval_us", "host_gen_us"}.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dcf_amd  # noqa: E402


def per_call(fn, n):
    for _ in range(max(3, n // 10)):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    rng = np.random.default_rng(1)
    prg = dcf_amd.Aes256HirosePrg([rng.bytes(32) for _ in range(2)], 16)
    d = dcf_amd.DcfImpl(16, 16, prg)
    k = d.gen(dcf_amd.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf_amd.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, 16, 16), np.uint8).copy()).cuda()
    s0 = torch.from_numpy(np.frombuffer(k.s0s[0], np.uint8).copy()).cuda()
    ev = {}
    for m in (1, 16, 128, 512, 2048, 8192, 32768, 65536, 100_000):
        xs = torch.randint(0, 256, (m, 16), dtype=torch.uint8, device="cuda")
        ys = torch.empty((m, 16), dtype=torch.uint8, device="cuda")
        ev[m] = per_call(lambda: d.eval_device(False, cwb, s0, xs, ys), 200 if m < 10000 else 50)
    gn = {}
    for K in (1, 16, 64, 256, 1024, 4096, 16384, 65536):
        a = torch.randint(0, 256, (K, 16), dtype=torch.uint8, device="cuda")
        b, c, e = (torch.randint(0, 256, (K, 16), dtype=torch.uint8, device="cuda") for _ in range(3))
        out = torch.empty(dcf_amd.cwb_bytes(16, 16, K), dtype=torch.uint8, device="cuda")
        gn[K] = per_call(lambda: d.gen_batch_device(a, b, c, e, dcf_amd.BoundState.LtBeta, out), 200)
    x1 = [rng.bytes(16)]
    share0 = dcf_amd.Share([k.s0s[0]], k.cws, k.cw_np1)
    host_eval = per_call(lambda: d.eval(False, share0, x1), 300)
    f = dcf_amd.CmpFn(rng.bytes(16), rng.bytes(16))
    host_gen = per_call(lambda: d.gen(f, [rng.bytes(16), rng.bytes(16)], dcf_amd.BoundState.LtBeta), 300)
    print(json.dumps({"lib": os.environ.get("DCF_HIP_LIB", "default"), "eval_us": ev, "gen_us": gn,
                      "host_eval_us": host_eval, "host_gen_us": host_gen}), flush=True)


if __name__ == "__main__":
    main()
