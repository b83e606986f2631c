"""Per-call time of device-resident single-key evals around DCF_EVAL_ROW_MAX (k_eval16_row vs
k_eval16_oct), around DCF_EVAL_ROW2_MAX (`small`: k_eval16_row2 vs k_eval16_row) and of batched gens
around DCF_GEN_ROW_MAX (k_gen16_row vs k_gen16_col):
DCF_HIP_LIB=... python scripts/row_threshold.py [gen|small] -> one JSON line {m: us}."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dcf_amd  # noqa: E402


def main():
    rng = np.random.default_rng(1)
    prg = dcf_amd.Aes256HirosePrg([rng.bytes(32) for _ in range(2)], 16)
    d = dcf_amd.DcfImpl(16, 16, prg)
    k = d.gen(dcf_amd.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf_amd.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, 16, 16), np.uint8).copy()).cuda()
    s0 = torch.from_numpy(np.frombuffer(k.s0s[0], np.uint8).copy()).cuda()
    out = {}
    if len(sys.argv) > 1 and sys.argv[1] == "gen":
        for K in (512, 1024, 2048, 4096, 8192):
            a, b, c, e = (torch.randint(0, 256, (K, 16), dtype=torch.uint8, device="cuda") for _ in range(4))
            o = torch.empty(dcf_amd.cwb_bytes(16, 16, K), dtype=torch.uint8, device="cuda")
            for _ in range(20):
                d.gen_batch_device(a, b, c, e, dcf_amd.BoundState.LtBeta, o)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(200):
                d.gen_batch_device(a, b, c, e, dcf_amd.BoundState.LtBeta, o)
                torch.cuda.synchronize()
            out[K] = (time.perf_counter() - t0) / 200 * 1e6
        print(json.dumps({"lib": os.environ.get("DCF_HIP_LIB", "default"), "gen_us": out}), flush=True)
        return
    sizes = (4096, 8192, 12000, 16384, 24576, 32768)
    if len(sys.argv) > 1 and sys.argv[1] == "small":  # around DCF_EVAL_ROW2_MAX (k_eval16_row2 vs k_eval16_row)
        sizes = (1, 4, 16, 64, 128, 256, 512, 1024, 2048, 4096)
    for m in sizes:
        xs = torch.randint(0, 256, (m, 16), dtype=torch.uint8, device="cuda")
        ys = torch.empty((m, 16), dtype=torch.uint8, device="cuda")
        for _ in range(20):
            d.eval_device(False, cwb, s0, xs, ys)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            d.eval_device(False, cwb, s0, xs, ys)
            torch.cuda.synchronize()
        out[m] = (time.perf_counter() - t0) / 200 * 1e6
    print(json.dumps({"lib": os.environ.get("DCF_HIP_LIB", "default"), "eval_us": out}), flush=True)


if __name__ == "__main__":
    main()
