"""Debug aid: which latency path differs from the oracle, and how (first differing bytes)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dcf_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402


def T(b):
    return torch.from_numpy(np.frombuffer(bytes(b), np.uint8).copy()).cuda()


def main():
    rng = np.random.default_rng(5)
    nb = 2
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf_amd.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    d = dcf_amd.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    n = 8 * nb
    # gen, device path (k_gen16_col, K = 1)
    A = T(alpha).view(1, nb)
    cwb = d.gen_batch_device(A, T(beta).view(1, 16), T(s0).view(1, 16), T(s1).view(1, 16), dcf_amd.BoundState.LtBeta)
    torch.cuda.synchronize()
    c = cwb.cpu().numpy()
    print("gen dev cw_s", np.array_equal(c[:n * 16].reshape(n, 16), ok.cw_s), c[:16].tobytes().hex(), bytes(ok.cw_s[0]).hex())
    print("gen dev cw_v", np.array_equal(c[n * 16:2 * n * 16].reshape(n, 16), ok.cw_v), c[n*16:n*16+16].tobytes().hex(), bytes(ok.cw_v[0]).hex())
    print("gen dev cw_t", list(c[2 * n * 16:2 * n * 16 + n]), list(ok.cw_t))
    k = d.gen(dcf_amd.CmpFn(alpha, beta), [s0, s1], dcf_amd.BoundState.LtBeta)
    print("gen host cw_s", [cw.s for cw in k.cws] == [bytes(r) for r in ok.cw_s], k.cws[0].s.hex())
    print("gen host t", [int(cw.tl) | int(cw.tr) << 1 for cw in k.cws], list(ok.cw_t))
    # eval with the oracle's key
    kk = dcf_amd.Share([s0], [dcf_amd.Cw(bytes(ok.cw_s[i]), bytes(ok.cw_v[i]), bool(ok.cw_t[i] & 1), bool(ok.cw_t[i] & 2))
                             for i in range(n)], bytes(ok.cw_np1))
    xs = rng.integers(0, 256, (5, nb), dtype=np.uint8)
    want = O.eval_(P, 0, ok, s0, xs)
    got = d.eval(False, kk, xs)
    print("eval host", np.array_equal(got, want))
    for i in range(5):
        print("  ", got[i].tobytes().hex(), want[i].tobytes().hex())
    yd = d.eval_device(False, T(dcf_amd.share_to_cwb(kk, nb, 16)), T(s0), torch.from_numpy(xs).cuda())
    torch.cuda.synchronize()
    print("eval dev", np.array_equal(yd.cpu().numpy(), want))
    for i in range(5):
        print("  ", yd[i].cpu().numpy().tobytes().hex())
    prg.set_eval_mode(4)
    yd = d.eval_device(False, T(dcf_amd.share_to_cwb(kk, nb, 16)), T(s0), torch.from_numpy(xs).cuda())
    torch.cuda.synchronize()
    print("eval dev stream engine", np.array_equal(yd.cpu().numpy(), want))


if __name__ == "__main__":
    main()
