"""Batched multi-key LAMBDA >= 32 eval vs one head/tail pipeline per key (the round-3 path):
K keys x P points, N = 16, one party; the per-key figure calls eval_device once per key on the
same buffers (what eval_body did for every key before r04).  Prints one JSON line.

  python scripts/wide_mk_bench.py [lam] [K] [P]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dcf_amd  # noqa: E402


def main():
    lam = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    nb = 16
    rng = np.random.default_rng(7)
    prg = dcf_amd.Aes256HirosePrg([rng.bytes(32) for _ in range(18)], lam)
    d = dcf_amd.DcfImpl(nb, lam, prg)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    r = lambda *s: rng.integers(0, 256, s, dtype=np.uint8)  # noqa: E731
    alpha, beta, s0, s1 = r(K, nb), r(K, lam), r(K, lam), r(K, lam)
    cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf_amd.BoundState.LtBeta)
    xs = T(r(K * P, nb))
    s0d = T(s0)
    ys = torch.empty((K * P, lam), dtype=torch.uint8, device="cuda")

    def batched():
        d.eval_multikey_device(False, cwb, s0d, xs, P, ys)

    # per key: that key's CWB (the single-key layout) and points, as the per-key path ran them
    cw = cwb.cpu().numpy()
    n = 8 * nb
    cws = cw[:n * K * lam].reshape(n, K, lam)
    cwv = cw[n * K * lam:2 * n * K * lam].reshape(n, K, lam)
    cwt = cw[2 * n * K * lam:2 * n * K * lam + n * K].reshape(n, K)
    off = dcf_amd.cwb_np1_offset(nb, lam, K)
    np1 = cw[off:off + K * lam].reshape(K, lam)
    one = dcf_amd.cwb_bytes(nb, lam, 1)
    o1 = dcf_amd.cwb_np1_offset(nb, lam, 1)
    keys = []
    for k in range(min(K, 512)):
        b = np.zeros(one, np.uint8)
        b[:n * lam] = cws[:, k].reshape(-1)
        b[n * lam:2 * n * lam] = cwv[:, k].reshape(-1)
        b[2 * n * lam:2 * n * lam + n] = cwt[:, k]
        b[o1:o1 + lam] = np1[k]
        keys.append(T(b))
    nk = len(keys)
    yk = torch.empty((nk * P, lam), dtype=torch.uint8, device="cuda")

    def per_key():
        for k in range(nk):
            d.eval_device(False, keys[k], s0d[k], xs[k * P:(k + 1) * P], yk[k * P:(k + 1) * P])

    def timeit(f, reps):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    tb = timeit(batched, 5)
    tp = timeit(per_key, 2)
    per_key_equal = bool(torch.equal(ys[:nk * P], yk))
    print(json.dumps({"lambda": lam, "keys": K, "points_per_key": P, "n_bytes": nb,
                      "batched_ms": tb * 1e3, "batched_evals_per_s": K * P / tb,
                      "per_key_ms_for_keys": tp * 1e3, "per_key_keys": nk, "per_key_evals_per_s": nk * P / tp,
                      "speedup": (K * P / tb) / (nk * P / tp), "outputs_equal": per_key_equal}), flush=True)


if __name__ == "__main__":
    main()
