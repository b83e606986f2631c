"""GPU parity: the HIP path (through the C ABI) against the golden vectors and
the CPU oracle, bit for bit.  Runs on an MI355X only (`-m gpu`)."""
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden.make_golden import REF_ALPHAS, REF_BETA, REF_KEYS, detbytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dcf(hip_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import dcf_amd
    return dcf_amd


def _rand(rng, shape):
    return rng.integers(0, 256, size=shape, dtype=np.uint8)


def test_prg16_golden(dcf, golden):
    g = golden("prg16")
    prg = dcf.Aes256HirosePrg([bytes.fromhex(k) for k in g["keys"]], 16)
    outs = prg.gen_many([bytes.fromhex(r["seed"]) for r in g["rows"]])
    for r, ((sl, vl, tl), (sr, vr, tr)) in zip(g["rows"], outs):
        assert (sl.hex(), vl.hex(), tl, sr.hex(), vr.hex(), tr) == (r["sl"], r["vl"], r["tl"], r["sr"], r["vr"],
                                                                      r["tr"])


def _full_cases(golden):
    return [c for c in golden("dcf_cases") if "keys" in c]


def test_prg32_golden(dcf, golden):
    g = golden("prg32")
    prg = dcf.Aes256HirosePrg([bytes.fromhex(k) for k in g["keys"]], 32)
    outs = prg.gen_many([bytes.fromhex(r["seed"]) for r in g["rows"]])
    for r, ((sl, vl, tl), (sr, vr, tr)) in zip(g["rows"], outs):
        assert (sl.hex(), vl.hex(), tl, sr.hex(), vr.hex(), tr) == (r["sl"], r["vl"], r["tl"], r["sr"], r["vr"],
                                                                      r["tr"])


@pytest.mark.parametrize("lam,nkeys", [(48, 18), (64, 20), (256, 18)])
def test_prg_wide_vs_oracle(dcf, lam, nkeys):
    rng = np.random.default_rng(lam)
    keys = [rng.bytes(32) for _ in range(nkeys)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    seeds = [rng.bytes(lam) for _ in range(9)]
    assert prg.gen_many(seeds) == [P.gen(s) for s in seeds]


def test_gen_golden(dcf, golden):
    for c in _full_cases(golden):
        lam = c["lambda"]
        prg = dcf.Aes256HirosePrg([bytes.fromhex(k) for k in c["keys"]], lam)
        d = dcf.DcfImpl(c["n_bytes"], lam, prg)
        s0s = [bytes.fromhex(s) for s in c["s0s"]]
        k = d.gen(dcf.CmpFn(bytes.fromhex(c["alpha"]), bytes.fromhex(c["beta"])), s0s, dcf.BoundState(c["bound"]))
        assert dcf.share_to_cwb(k, c["n_bytes"], lam).hex() == c["cwb"], c["name"]


def test_large_lambda_golden(dcf, golden):
    """benches/dcf_large_lambda.rs shape (LAMBDA = 16384, 2048 AES keys) at N = 2."""
    for c in golden("dcf_cases"):
        if "keys" in c:
            continue
        lam, nb = c["lambda"], c["n_bytes"]
        keys = [detbytes(c["keys_fmt"].format(i=i), 32) for i in range(c["cipher_n"])]
        prg = dcf.Aes256HirosePrg(keys, lam)
        d = dcf.DcfImpl(nb, lam, prg)
        s0s = [detbytes(t, lam) for t in c["s0_tags"]]
        k = d.gen(dcf.CmpFn(detbytes(c["alpha_tag"], nb), detbytes(c["beta_tag"], lam)), s0s,
                  dcf.BoundState(c["bound"]))
        assert hashlib.sha256(dcf.share_to_cwb(k, nb, lam)).hexdigest() == c["cwb_sha256"]
        xs = [detbytes(c["xs_fmt"].format(i=i), nb) for i in range(c["m"])]
        for b, key in ((0, "y0_sha256"), (1, "y1_sha256")):
            ys = d.eval(bool(b), dcf.Share([s0s[b]], k.cws, k.cw_np1), xs)
            assert hashlib.sha256(ys.tobytes()).hexdigest() == c[key], (c["name"], b)


def test_eval_golden(dcf, golden):
    for c in _full_cases(golden):
        lam = c["lambda"]
        prg = dcf.Aes256HirosePrg([bytes.fromhex(k) for k in c["keys"]], lam)
        nb = c["n_bytes"]
        d = dcf.DcfImpl(nb, lam, prg)
        s0s = [bytes.fromhex(s) for s in c["s0s"]]
        full = dcf.cwb_to_share(bytes.fromhex(c["cwb"]), nb, lam, s0s)
        xs = [bytes.fromhex(x) for x in c["xs"]]
        for b, key in ((0, "y0"), (1, "y1")):
            k = dcf.Share([s0s[b]], full.cws, full.cw_np1)  # lib.rs:382-385: s0s trimmed per party
            ys = d.eval(bool(b), k, xs)
            assert [y.tobytes().hex() for y in ys] == c[key], (c["name"], b)


@pytest.mark.parametrize("bound", [0, 1])
def test_reference_reconstruction_kat(dcf, bound):
    """lib.rs:372-420 and 422-442 on the GPU, seeds fixed."""
    prg = dcf.Aes256HirosePrg(REF_KEYS, 16)
    d = dcf.DcfImpl(16, 16, prg)
    expect = [1, 1, 0, 0, 0] if bound == 0 else [0, 0, 0, 1, 1]
    for trial in range(3):
        s0s = [detbytes(f"gkat/{trial}/0", 16), detbytes(f"gkat/{trial}/1", 16)]
        k = d.gen(dcf.CmpFn(REF_ALPHAS[2], REF_BETA), s0s, dcf.BoundState(bound))
        y0 = d.eval(False, dcf.Share([s0s[0]], k.cws, k.cw_np1), REF_ALPHAS)
        y1 = d.eval(True, dcf.Share([s0s[1]], k.cws, k.cw_np1), REF_ALPHAS)
        for i, e in enumerate(expect):
            assert (y0[i] ^ y1[i]).tobytes() == (REF_BETA if e else bytes(16))
        assert y0[2].tobytes() != bytes(16) and y1[2].tobytes() != bytes(16)


@pytest.mark.parametrize("mode", [0, 1, 4])
@pytest.mark.parametrize("nb", [1, 2, 3, 4, 5, 7, 8, 12, 16, 17, 32])
def test_eval_random_vs_oracle(dcf, nb, mode):
    """mode 0 = auto, 1 = lockstep LDS T-table engine (k_eval16, also for one key), 4 = T-table
    with per-lane block scheduling (stream engine)."""
    rng = np.random.default_rng(100 + nb)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    prg.set_eval_mode(mode)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    ok = O.gen(P, alpha, beta, s0, s1, int(nb % 2))
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(nb % 2))
    cwb = dcf.share_to_cwb(k, nb, 16)
    raw = ok.cw_s.tobytes() + ok.cw_v.tobytes() + ok.cw_t.tobytes()
    assert cwb == raw + bytes((-len(raw)) % 16) + ok.cw_np1.tobytes()
    for m in (0, 1, 31, 33, 63, 64, 65, 513, 777):
        xs = _rand(rng, (m, nb))
        if m > 3:
            xs[0] = np.frombuffer(alpha, np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            want = O.eval_(P, b, ok, s, xs, nthreads=4)
            assert np.array_equal(got, want), (nb, m, b)


@pytest.mark.parametrize("nb,levels", [(1, 1), (1, 7), (2, 9), (2, 15), (3, 23), (4, 8), (4, 24), (5, 1),
                                        (16, 13), (16, 24), (17, 20), (32, 24), (4, 26), (32, 30),
                                        (4, 19), (4, 21), (16, 22)])
def test_eval_prefix_table_vs_oracle(dcf, nb, levels):
    """Shared-prefix eval (stream engine, forced depth): points start at level D from
    the key's expanded top tree; the output must not change.  Covers D = 1, D = 8N - 1
    (the walk's last level only), D across x's word boundary (N = 3: 24 bits) and
    the 28-level cap on a forced depth (N = 32, D = 30); D = 19 / 20 / 21 / 22+ build the
    last 1 / 2 / 3 / 4 levels depth-first (k_prefix_build16 tail)."""
    rng = np.random.default_rng(700 + 31 * nb + levels)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    prg.set_eval_mode(4)
    prg.set_prefix_levels(levels)
    want_d = min(levels, 28, 8 * nb - 1)
    m = 3001
    assert prg.eval_prefix_levels(nb, 1, m) == want_d
    d = dcf.DcfImpl(nb, 16, prg)
    for bound in (0, 1):
        alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        xs = _rand(rng, (m, nb))
        a = np.frombuffer(alpha, np.uint8)
        xs[0] = a
        xs[1] = 0
        xs[2] = 255
        xs[3:40] = a  # points sharing alpha's prefix, differing in the last byte
        xs[3:40, -1] = rng.integers(0, 256, 37, dtype=np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            want = O.eval_(P, b, ok, s, xs, nthreads=8)
            assert np.array_equal(got, want), (nb, levels, bound, b)
    prg.set_prefix_levels(0)
    assert prg.eval_prefix_levels(nb, 1, m) == 0
    prg.set_prefix_levels(-1)
    assert prg.eval_prefix_levels(16, 1, 1 << 28) == 27  # auto: log2(points), capped
    assert prg.eval_prefix_levels(16, 1, 1 << 20) == 20
    assert prg.eval_prefix_levels(2, 1, 1 << 20) == 15   # < 8N
    assert prg.eval_prefix_levels(16, 2, 1 << 20) == 0   # one key only
    with pytest.raises(dcf.DcfError):
        prg.set_prefix_levels(-2)


def test_eval_length_mismatch_is_error(dcf):
    prg = dcf.Aes256HirosePrg(REF_KEYS, 16)
    d = dcf.DcfImpl(16, 16, prg)
    k = d.gen(dcf.CmpFn(REF_ALPHAS[0], REF_BETA), [bytes(16), bytes(16)], dcf.BoundState.LtBeta)
    with pytest.raises(dcf.DcfError):
        d.eval(False, k, REF_ALPHAS, np.zeros((4, 16), np.uint8))  # reference would silently truncate
    with pytest.raises(dcf.DcfError):
        d.eval(False, dcf.Share(k.s0s, k.cws[:127], k.cw_np1), REF_ALPHAS)  # lib.rs:165


@pytest.mark.parametrize("mode", [1, 4])
@pytest.mark.parametrize("nb,m", [(16, 1 << 20), (4, (1 << 20) + 37)])
def test_eval_device_large_sample_and_reconstruction(dcf, nb, m, mode):
    """Large batch on device: bit-exact on a sample vs the oracle, and the
    reconstruction property y0 ^ y1 == beta * [x < alpha] on every point."""
    import torch
    rng = np.random.default_rng(nb)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    prg.set_eval_mode(mode)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf.share_to_cwb(k, nb, 16), np.uint8).copy()).cuda()
    xs_h = _rand(rng, (m, nb))
    xs = torch.from_numpy(xs_h).cuda()
    y0 = d.eval_device(False, cwb, torch.tensor(list(s0), dtype=torch.uint8).cuda(), xs)
    y1 = d.eval_device(True, cwb, torch.tensor(list(s1), dtype=torch.uint8).cuda(), xs)
    torch.cuda.synchronize()
    y0h, y1h = y0.cpu().numpy(), y1.cpu().numpy()
    idx = np.unique(np.concatenate([np.arange(64), np.arange(m - 64, m), rng.integers(0, m, 512)]))
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    assert np.array_equal(y0h[idx], O.eval_(P, 0, ok, s0, xs_h[idx], nthreads=8))
    assert np.array_equal(y1h[idx], O.eval_(P, 1, ok, s1, xs_h[idx], nthreads=8))
    # reconstruction on all points, vectorised: lexicographic x < alpha on big-endian bytes
    a = np.frombuffer(alpha, np.uint8)
    diff = xs_h != a
    first = np.where(diff.any(1), diff.argmax(1), nb)
    lt = np.zeros(m, bool)
    has = first < nb
    lt[has] = xs_h[has, first[has]] < a[first[has]]
    rec = y0h ^ y1h
    bt = np.frombuffer(beta, np.uint8)
    assert np.array_equal(rec[lt], np.broadcast_to(bt, (int(lt.sum()), 16)))
    assert not rec[~lt].any()


@pytest.mark.parametrize("nb,K,P", [(1, 70, 64), (3, 130, 40), (4, 70, 64), (4, 130, 32), (4, 65, 48), (5, 65, 33),
                                     (16, 200, 32), (17, 40, 48), (32, 70, 40)])
def test_multikey_stream_widths_vs_oracle(dcf, nb, K, P):
    """Multi-key stream eval (per-key top trees, key-major CW digest) at 8N levels that are not a
    multiple of the digest's 16-level tiles and key counts that are not a multiple of 64."""
    import torch
    rng = np.random.default_rng(nb * 7919 + K)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, Po = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    prg.set_eval_mode(4)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = (_rand(rng, (K, nb)), _rand(rng, (K, 16)), _rand(rng, (K, 16)), _rand(rng, (K, 16)))
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf.BoundState(0))
    xs = _rand(rng, (K * P, nb))
    y0 = d.eval_multikey_device(False, cwb, T(s0), T(xs), P)
    y1 = d.eval_multikey_device(True, cwb, T(s1), T(xs), P)
    torch.cuda.synchronize()
    y0h, y1h = y0.cpu().numpy(), y1.cpu().numpy()
    for key in sorted(set([0, K - 1] + list(rng.integers(0, K, 5)))):
        ok = O.gen(Po, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), 0)
        sl = slice(key * P, (key + 1) * P)
        assert np.array_equal(y0h[sl], O.eval_(Po, 0, ok, s0[key].tobytes(), xs[sl]))
        assert np.array_equal(y1h[sl], O.eval_(Po, 1, ok, s1[key].tobytes(), xs[sl]))


@pytest.mark.parametrize("mode", [0, 1, 4])
@pytest.mark.parametrize("K,P", [(1, 100), (37, 64), (10, 13), (300, 128)])
def test_gen_batch_and_multikey_eval_vs_oracle(dcf, K, P, mode):
    """mode 0 (auto) on these small batches runs the two-lanes-per-point lockstep kernel
    (k_eval16_pair) in all three key modes: one key, keys wave-uniform (P % 64 == 0), any P."""
    import torch
    nb = 16
    rng = np.random.default_rng(K * 1000 + P)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, Po = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    prg.set_eval_mode(mode)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = (_rand(rng, (K, nb)), _rand(rng, (K, 16)), _rand(rng, (K, 16)), _rand(rng, (K, 16)))
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    for bound in (0, 1):
        cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf.BoundState(bound))
        xs = _rand(rng, (K * P, nb))
        xs[::P] = alpha  # x == alpha for the first point of each key
        y0 = d.eval_multikey_device(False, cwb, T(s0), T(xs), P)
        y1 = d.eval_multikey_device(True, cwb, T(s1), T(xs), P)
        torch.cuda.synchronize()
        cw = cwb.cpu().numpy()
        n = 8 * nb
        cws = cw[:n * K * 16].reshape(n, K, 16)
        cwv = cw[n * K * 16:2 * n * K * 16].reshape(n, K, 16)
        cwt = cw[2 * n * K * 16:2 * n * K * 16 + n * K].reshape(n, K)
        off = dcf.cwb_np1_offset(nb, 16, K)
        np1 = cw[off:off + K * 16].reshape(K, 16)
        y0h, y1h = y0.cpu().numpy(), y1.cpu().numpy()
        for key in sorted(set([0, K - 1] + list(rng.integers(0, K, 6)))):
            ok = O.gen(Po, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), bound)
            assert np.array_equal(cws[:, key], ok.cw_s) and np.array_equal(cwv[:, key], ok.cw_v)
            assert np.array_equal(cwt[:, key], ok.cw_t) and np.array_equal(np1[key], ok.cw_np1)
            sl = slice(key * P, (key + 1) * P)
            assert np.array_equal(y0h[sl], O.eval_(Po, 0, ok, s0[key].tobytes(), xs[sl]))
            assert np.array_equal(y1h[sl], O.eval_(Po, 1, ok, s1[key].tobytes(), xs[sl]))
        # reconstruction at x == alpha is 0 for both bounds (f(alpha) = 0, lib.rs:62)
        assert not (y0h[::P] ^ y1h[::P]).any()


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("lam,nb,m", [(32, 2, 70), (48, 3, 65), (64, 16, 33), (112, 4, 130), (1024, 2, 40),
                                      (4096, 16, 12), (272, 5, 600), (512, 16, 5000), (16384, 16, 150)])
def test_wide_eval_random_vs_oracle(dcf, lam, nb, m, mode):
    """LAMBDA >= 32: head/tail kernels vs the literal oracle, both parties, both bounds.
    mode 0: stream head (default), mode 1: lockstep T-table head.  LAMBDA % 128 == 0 runs the
    paired-slot tail (k_eval_wide_tail2), (64, 16) the compile-time 33-chunk 4-bit tail and
    (48, 3), (112, 4), (272, 5) the runtime-chunk one; 16384 covers 128 tiles per point."""
    rng = np.random.default_rng(lam * 7 + nb)
    keys = [rng.bytes(32) for _ in range(18)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    prg.set_eval_mode(mode)
    d = dcf.DcfImpl(nb, lam, prg)
    for bound in (0, 1):
        alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        raw = ok.cw_s.tobytes() + ok.cw_v.tobytes() + ok.cw_t.tobytes()
        assert dcf.share_to_cwb(k, nb, lam) == raw + bytes((-len(raw)) % 16) + ok.cw_np1.tobytes()
        xs = _rand(rng, (m, nb))
        xs[0] = np.frombuffer(alpha, np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), (lam, nb, b, bound)


def _small_auto_depth(nb, m):
    """Auto depth on the small-batch path (dcf_hip.hip small_prefix_depth): none up to 32768
    points (the latency kernels' sizes; at N > 32 the pair walk without a table), else 18 below
    2^18 points and 19 from there, at most 8N - 1, none below 8."""
    if m <= 32768:
        return 0
    d = min(18 if m < (1 << 18) else 19, 8 * nb - 1)
    return d if d >= 8 else 0


@pytest.mark.parametrize("nb,levels,m", [(16, 9, 3000), (16, 15, 20000), (16, 31, 5000), (4, 12, 4000), (3, 23, 2000),
                                         (1, 5, 700), (5, 33, 1500), (16, -1, 20000), (2, -1, 40000),
                                         (16, -1, 100000), (4, -1, 300000), (1, -1, 50000), (33, -1, 3000)])
def test_small_pair_prefix_vs_oracle(dcf, nb, levels, m):
    """Small batches (auto engine: the two-lanes-per-point path, k_eval16_pair) below a
    shared-prefix table: forced depths (D = 5 .. 31, x-word boundary at N = 3, 5) and the auto
    depth (-1: 18 / 19, capped at 8N - 1; none on the latency kernels' sizes, nor at N = 1);
    both parties and bounds, vs the oracle."""
    rng = np.random.default_rng(4000 + 37 * nb + levels)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    prg.set_prefix_levels(levels)
    want_d = min(levels, 28, 8 * nb - 1) if levels > 0 else _small_auto_depth(nb, m)
    assert prg.eval_prefix_levels(nb, 1, m) == want_d
    d = dcf.DcfImpl(nb, 16, prg)
    for bound in (0, 1):
        alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        xs = _rand(rng, (m, nb))
        a = np.frombuffer(alpha, np.uint8)
        xs[0] = a
        xs[3:40] = a
        xs[3:40, -1] = rng.integers(0, 256, 37, dtype=np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), (nb, levels, m, bound, b)


@pytest.mark.parametrize("lam,nb,m", [(128, 1, 300), (256, 3, 200), (128, 4, 500), (384, 6, 300), (128, 8, 40000),
                                      (256, 12, 150), (128, 16, 33000), (256, 5, 100), (128, 9, 300),
                                      (256, 10, 200), (128, 11, 40000), (384, 13, 200), (128, 14, 300),
                                      (256, 15, 500), (128, 2, 300), (256, 7, 200), (128, 17, 200)])
def test_wide_tail2_layouts_vs_oracle(dcf, lam, nb, m):
    """The paired-slot tail (k_eval_wide_tail2, LAMBDA % 128 == 0) in every instantiated chunk
    layout, row 0 (t_0 = party) folded into the constant (r05): N = 1 (0,1), 2 and 3 (2,0), 4
    (1,2), 5 and 6 (4,0), 7 (3,2), 8 and 9 (6,0), 10 (5,2), 11 and 12 (8,0), 13 (7,2), 14 and 15
    (10,0) and 16 (9,2) (both LDS-filling: global block counters), 17 (8,4); 40000 / 33000 points
    cross the 32768-point workgroup ranges, and the t-vector repack (k_tvec_chunks) runs in place
    on the head's rows.  Both parties: party 1 takes the folded row, party 0 not."""
    rng = np.random.default_rng(lam * 13 + nb)
    keys = [rng.bytes(32) for _ in range(18)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    for bound in (0, 1):
        alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        xs = _rand(rng, (m, nb))
        xs[0] = np.frombuffer(alpha, np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), (lam, nb, b, bound)


@pytest.mark.parametrize("lam,nb,depth,m", [(32, 2, 1, 300), (32, 4, 16, 3000), (64, 16, 8, 2000), (48, 3, 23, 700),
                                            (272, 5, 17, 2500), (16384, 16, 15, 120), (16384, 16, 21, 64), (64, 4, 15, 900),
                                            (128, 2, 30, 500), (64, 16, -1, 1100)])
def test_wide_prefix_vs_oracle(dcf, lam, nb, depth, m):
    """LAMBDA >= 32 stream head below a shared-prefix table (k_wpfx_level: bytes [0,32)
    of the walk for the top D levels, with t-vector rows 0..D): bit-exact with the oracle
    for D = 1, 8 (partial t-vector word), 15 (word 0 completed by the table's last
    level), 16 and 17 (word 0 complete, word 1 partial at start), 21,
    23, D capped at 8N - 1 (N = 2, D = 30), auto (-1: 2^10 points -> 9), lambda = 32
    (the cleared bit inside the head's bytes), both parties and bounds."""
    rng = np.random.default_rng(lam + 31 * nb + depth)
    keys = [rng.bytes(32) for _ in range(18)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    prg.set_prefix_levels(depth)
    want_d = min(8 * nb - 1, 30, depth) if depth > 0 else min(8 * nb - 1, 22, int(np.log2(m)) - 1)
    assert prg.eval_prefix_levels(nb, 1, m) == want_d
    d = dcf.DcfImpl(nb, lam, prg)
    for bound in (0, 1):
        alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        xs = _rand(rng, (m, nb))
        a = np.frombuffer(alpha, np.uint8)
        xs[0] = a
        xs[1:20] = a
        xs[1:20, -1] = rng.integers(0, 256, 19, dtype=np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), (lam, nb, depth, b, bound)
    prg.set_eval_mode(1)  # LAMBDA >= 32 has one head engine: the setting changes nothing
    assert prg.eval_prefix_levels(nb, 1, m) == want_d
    prg.set_prefix_levels(0)
    assert prg.eval_prefix_levels(nb, 1, m) == 0


def test_wide_gen_batch_and_multikey(dcf):
    import torch
    lam, nb, K, Pp = 64, 2, 5, 7
    rng = np.random.default_rng(99)
    keys = [rng.bytes(32) for _ in range(18)]
    prg, Po = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = (_rand(rng, (K, nb)), _rand(rng, (K, lam)), _rand(rng, (K, lam)), _rand(rng, (K, lam)))
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf.BoundState.GtBeta)
    xs = _rand(rng, (K * Pp, nb))
    y1 = d.eval_multikey_device(True, cwb, T(s1), T(xs), Pp)
    torch.cuda.synchronize()
    cw, y1h = cwb.cpu().numpy(), y1.cpu().numpy()
    n = 8 * nb
    cws = cw[:n * K * lam].reshape(n, K, lam)
    for key in range(K):
        ok = O.gen(Po, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), 1)
        assert np.array_equal(cws[:, key], ok.cw_s)
        sl = slice(key * Pp, (key + 1) * Pp)
        assert np.array_equal(y1h[sl], O.eval_(Po, 1, ok, s1[key].tobytes(), xs[sl]))


@pytest.mark.parametrize("lam,nb,K,P", [(32, 2, 9, 5), (64, 3, 40, 17), (96, 2, 12, 33), (128, 16, 70, 64),
                                         (256, 5, 300, 8), (128, 40, 20, 30), (96, 3, 4, 9000), (32, 2, 5000, 8),
                                         (128, 4, 3, 40000), (64, 170, 4, 9)])
def test_wide_multikey_batched_vs_oracle(dcf, lam, nb, K, P):
    """LAMBDA >= 32 multi-key eval: keys with <= 32768 points go through batched head / tail
    passes of up to 4096 keys (per-point key, per-workgroup key tables; the 4-bit tail at
    LAMBDA = 96 — with 9000 points per key, three tail ranges per key — and at N = 40, the
    paired-slot tail at 128 / 256; 5000 keys take two passes; N = 170, two tail passes over the
    t-sequence); 40000 points per key takes the per-key path.  Both parties reconstruct."""
    import torch
    rng = np.random.default_rng(lam * 31 + K)
    keys = [rng.bytes(32) for _ in range(18)]
    prg, Po = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = (_rand(rng, (K, nb)), _rand(rng, (K, lam)), _rand(rng, (K, lam)), _rand(rng, (K, lam)))
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf.BoundState.LtBeta)
    xs = _rand(rng, (K * P, nb))
    xs[::P] = alpha
    y0 = d.eval_multikey_device(False, cwb, T(s0), T(xs), P)
    y1 = d.eval_multikey_device(True, cwb, T(s1), T(xs), P)
    torch.cuda.synchronize()
    y0h, y1h = y0.cpu().numpy(), y1.cpu().numpy()
    for key in sorted(set([0, K - 1] + list(rng.integers(0, K, 4)))):
        ok = O.gen(Po, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), 0)
        sl = slice(key * P, (key + 1) * P)
        assert np.array_equal(y0h[sl], O.eval_(Po, 0, ok, s0[key].tobytes(), xs[sl], nthreads=8)), key
        assert np.array_equal(y1h[sl], O.eval_(Po, 1, ok, s1[key].tobytes(), xs[sl], nthreads=8)), key
    assert not (y0h[::P] ^ y1h[::P]).any()  # f(alpha) = 0 for every key
    # the batched passes build no shared-prefix table, and the depth hook says so;
    # a forced depth sends the keys through the per-key path, which builds one per key
    want = 0 if P <= 32768 else min(P.bit_length() - 2, 22, 8 * nb - 1)
    assert prg.eval_prefix_levels(nb, K, P) == (want if want >= 8 else 0)
    if K <= 40 and P < 32768 and 8 * nb > 6:
        prg.set_prefix_levels(6)
        assert prg.eval_prefix_levels(nb, K, P) == 6
        y0f = d.eval_multikey_device(False, cwb, T(s0), T(xs), P)
        torch.cuda.synchronize()
        assert np.array_equal(y0f.cpu().numpy(), y0h)


@pytest.mark.parametrize("nb", [1, 4, 5, 8, 16, 17, 32])
@pytest.mark.parametrize("prefix", [0, -1])
def test_stream_b_reuse_vs_oracle(dcf, nb, prefix):
    """Stream engine's B reuse (a right step at t = 0 keeps the seed, so the next level's
    B is known): runs of right steps (x bytes 0xFF, 0xFE, 0x7F), both parties (t starts
    at 0 and 1), a root seed with the masked bit set and clear, 32-level word boundaries
    (N = 5, 17, 32); bit-exact with the oracle.  The kernel's own block count must sit
    below the no-reuse count 8N + zeros(x) and above 8N - (levels it could skip)."""
    rng = np.random.default_rng(0xB0 + nb)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    prg.set_eval_mode(4)
    prg.set_prefix_levels(prefix)
    d = dcf.DcfImpl(nb, 16, prg)
    m = 600_000 if prefix else 20_000
    for bound, masked in ((0, True), (1, False)):
        alpha, beta = rng.bytes(nb), rng.bytes(16)
        s0, s1 = bytearray(rng.bytes(16)), bytearray(rng.bytes(16))
        for sd in (s0, s1):
            sd[15] = (sd[15] & 0xFE) | (0 if masked else 1)
        s0, s1 = bytes(s0), bytes(s1)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        xs = _rand(rng, (m, nb))
        xs[:1000] = 0xFF
        xs[1000:2000] = rng.choice(np.array([0xFF, 0xFE, 0x7F, 0xEF], np.uint8), size=(1000, nb))
        xs[2000] = np.frombuffer(alpha, np.uint8)
        for b, sd in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([sd], k.cws, k.cw_np1), xs)
            blocks = prg.last_eval_blocks()
            idx = np.r_[0:4000, m - 2000:m]
            want = O.eval_(P, b, ok, sd, xs[idx], nthreads=8)
            assert np.array_equal(got[idx], want), (nb, prefix, bound, b)
            if prefix == 0:
                zeros = int(np.unpackbits(xs).size - np.unpackbits(xs).sum())
                assert blocks < 8 * nb * m + zeros, (blocks, 8 * nb * m + zeros)
                assert blocks > 0.5 * (8 * nb * m + zeros)


def test_retired_eval_modes_rejected(dcf):
    """Modes 2, 3 and 5 (bitsliced, hybrid, stream-hybrid; retired in round 5 after losing every
    A/B) are refused with DCF_ERR_ARG, and the prg keeps its engine."""
    prg = dcf.Aes256HirosePrg(REF_KEYS, 16)
    for mode in (2, 3, 5, 6, -1):
        with pytest.raises(dcf.DcfError) as e:
            prg.set_eval_mode(mode)
        assert e.value.code == -1
    for mode in (0, 1, 4):
        prg.set_eval_mode(mode)
    assert not hasattr(prg, "set_hybrid_split") and not hasattr(prg, "set_stream_hybrid")


def test_error_codes_on_device(dcf):
    with pytest.raises(dcf.DcfError) as e:
        dcf.Aes256HirosePrg([bytes(32)] * 17, 32)
    assert e.value.code == -3
    with pytest.raises(dcf.DcfError) as e:
        dcf.Aes256HirosePrg([bytes(32)] * 2, 8)
    assert e.value.code == -2


@pytest.mark.parametrize("nb,lam", [(1, 16), (2, 16), (3, 16), (1, 32), (1, 64)])
def test_full_domain_eval_vs_oracle(dcf, nb, lam):
    """Full-domain eval (tree expansion) == pointwise oracle eval over every x.  N = 2 and 3 take
    the one-launch table build for the levels above the depth-first tail (D = 12 and 20)."""
    import torch
    rng = np.random.default_rng(nb * 100 + lam)
    keys = [rng.bytes(32) for _ in range(2 if lam == 16 else 18)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf.share_to_cwb(k, nb, lam), np.uint8).copy()).cuda()
    xs = np.array([list(i.to_bytes(nb, "big")) for i in range(1 << (8 * nb))], np.uint8)
    ys = []
    for b, s in ((0, s0), (1, s1)):
        y = d.eval_full_domain_device(bool(b), cwb, torch.from_numpy(np.frombuffer(s, np.uint8).copy()).cuda())
        torch.cuda.synchronize()
        yh = y.cpu().numpy()
        assert np.array_equal(yh, O.eval_(P, b, ok, s, xs, nthreads=8)), (nb, lam, b)
        ys.append(yh)
    a = int.from_bytes(alpha, "big")
    rec = ys[0] ^ ys[1]
    assert not rec[a:].any() and (rec[:a] == np.frombuffer(beta, np.uint8)).all()


@pytest.mark.parametrize("nb", [2, 16])
def test_gen_batch_large_counter_path(dcf, nb):
    """>= 2^19 keys: batched gen takes 64-key units from the work counter; the multi-key
    eval runs the stream engine over the key-major digest.  A sample of keys vs the oracle."""
    import torch
    K, P = 600_000 if nb == 2 else 540_000, 1
    rng = np.random.default_rng(4242 + nb)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, Po = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    d = dcf.DcfImpl(nb, 16, prg)
    g = torch.Generator(device="cuda")
    g.manual_seed(nb)
    r = lambda *s: torch.randint(0, 256, s, dtype=torch.uint8, device="cuda", generator=g)  # noqa: E731
    alpha, beta, s0, s1, xs = r(K, nb), r(K, 16), r(K, 16), r(K, 16), r(K * P, nb)
    cwb = d.gen_batch_device(alpha, beta, s0, s1, dcf.BoundState.LtBeta)
    y0 = d.eval_multikey_device(False, cwb, s0, xs, P)
    y1 = d.eval_multikey_device(True, cwb, s1, xs, P)
    torch.cuda.synchronize()
    n = 8 * nb
    cw = cwb.cpu().numpy()
    cws = cw[:n * K * 16].reshape(n, K, 16)
    A, B, S0, S1, X = (t.cpu().numpy() for t in (alpha, beta, s0, s1, xs))
    Y0, Y1 = y0.cpu().numpy(), y1.cpu().numpy()
    for key in sorted(set([0, K - 1] + list(rng.integers(0, K, 24)))):
        ok = O.gen(Po, A[key].tobytes(), B[key].tobytes(), S0[key].tobytes(), S1[key].tobytes(), 0)
        assert np.array_equal(cws[:, key], ok.cw_s), key
        assert np.array_equal(Y0[key:key + 1], O.eval_(Po, 0, ok, S0[key].tobytes(), X[key:key + 1]))
        assert np.array_equal(Y1[key:key + 1], O.eval_(Po, 1, ok, S1[key].tobytes(), X[key:key + 1]))
    # reconstruction on every key: y0 ^ y1 = beta * [x < alpha]
    diff = X != A
    first = np.where(diff.any(1), diff.argmax(1), nb)
    lt = np.zeros(K, bool)
    has = first < nb
    lt[has] = X[has, first[has]] < A[has, first[has]]
    rec = Y0 ^ Y1
    assert np.array_equal(rec[lt], B[lt]) and not rec[~lt].any()


@pytest.mark.parametrize("nb,lam,m,mode", [(31, 128, 64, 0), (32, 128, 64, 0), (32, 128, 700, 0), (48, 128, 700, 0),
                                             (48, 128, 300, 1), (64, 256, 600, 0), (100, 128, 200, 0),
                                             (159, 128, 96, 0)])
def test_wide_large_n_vs_oracle(dcf, nb, lam, m, mode):
    """LAMBDA >= 32 at large inputs (the reference takes any N, lib.rs:163-165): the t-vector grows
    past 64 B from N = 32 (8N + 1 > 256 rows), the 4-bit tail narrows its tiles to keep its tables
    in the LDS (128-byte tiles to N = 39, 64 to N = 79, 32 to N = 159).  Stream head (mode 0; with
    m >= 512 below a shared-prefix table) and lockstep head (mode 1), both parties vs the oracle,
    alpha itself among the points."""
    rng = np.random.default_rng(0x31 + nb + m)
    keys = [rng.bytes(32) for _ in range(18)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    prg.set_eval_mode(mode)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    raw = ok.cw_s.tobytes() + ok.cw_v.tobytes() + ok.cw_t.tobytes()
    assert dcf.share_to_cwb(k, nb, lam) == raw + bytes((-len(raw)) % 16) + ok.cw_np1.tobytes()
    xs = _rand(rng, (m, nb))
    xs[0] = np.frombuffer(alpha, np.uint8)
    xs[1] = xs[0]
    xs[1, -1] ^= 1  # a neighbour of alpha: differs in the last level only
    for b, s in ((0, s0), (1, s1)):
        got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
        assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), b


@pytest.mark.parametrize("nb,lam,m,mode", [(160, 128, 96, 0), (161, 64, 70, 1), (200, 256, 40, 0),
                                             (401, 128, 33, 0)])
def test_wide_n_past_one_table_set_vs_oracle(dcf, nb, lam, m, mode):
    """N >= 160 at LAMBDA >= 32: the t-sequence has more 4-row chunks (> 320) than one set of
    32-byte-tile tables holds in the LDS, so the tail runs in passes of 320 chunks, each after the
    first adding its rows' share to the y the previous pass wrote (N = 401: three passes, the last
    with 3 chunks).  Both parties vs the oracle, alpha and a neighbour among the points."""
    rng = np.random.default_rng(0x160 + nb + lam)
    keys = [rng.bytes(32) for _ in range(18)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    prg.set_eval_mode(mode)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    xs = _rand(rng, (m, nb))
    xs[0] = np.frombuffer(alpha, np.uint8)
    xs[1] = xs[0]
    xs[1, -1] ^= 1
    ys = []
    for b, s in ((0, s0), (1, s1)):
        got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
        assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), b
        ys.append(got)
    rec = ys[0] ^ ys[1]
    a = int.from_bytes(alpha, "big")
    for i in range(m):
        on = int.from_bytes(xs[i].tobytes(), "big") < a
        assert rec[i].tobytes() == (beta if on else bytes(lam)), i


@pytest.mark.parametrize("kind,lam,nb", [(0, 16, 16), (0, 128, 16), (0, 64, 200), (1, 16, 4), (1, 64, 40)])
def test_empty_batches_every_path(dcf, kind, lam, nb):
    """Empty inputs are no-ops on every entry point, both PRGs, LAMBDA = 16 and >= 32 (the
    reference's eval maps an empty xs to an empty ys, lib.rs:163-204): host eval of 0 points,
    device eval of 0 points, batched gen of 0 keys, multi-key eval of 0 keys and of K keys x 0
    points; a following non-empty eval on the same prg is still exact."""
    import torch
    rng = np.random.default_rng(kind * 1000 + lam + nb)
    if kind == 0:
        keys = [rng.bytes(32) for _ in range(18)]
        prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    else:
        keys = [rng.bytes(16) for _ in range(4 * lam // 16)]
        prg, P = dcf.Aes128MatyasMeyerOseasPrg(keys, lam), O.OracleMmoPrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    assert d.eval(False, dcf.Share([s0], k.cws, k.cw_np1), np.zeros((0, nb), np.uint8)).shape == (0, lam)
    dev = "cuda"
    cwb = torch.from_numpy(np.frombuffer(dcf.share_to_cwb(k, nb, lam), np.uint8).copy()).to(dev)
    s0d = torch.from_numpy(np.frombuffer(s0, np.uint8).copy()).to(dev)
    assert d.eval_device(False, cwb, s0d, torch.empty((0, nb), dtype=torch.uint8, device=dev)).shape == (0, lam)
    e = lambda *sh: torch.empty(sh, dtype=torch.uint8, device=dev)  # noqa: E731
    g0 = d.gen_batch_device(e(0, nb), e(0, lam), e(0, lam), e(0, lam), dcf.BoundState.LtBeta)
    assert g0.numel() == dcf.cwb_bytes(nb, lam, 0)
    assert d.eval_multikey_device(False, g0, e(0, lam), e(0, nb), 5).shape == (0, lam)
    K = 3
    r = lambda *sh: torch.from_numpy(rng.integers(0, 256, sh, dtype=np.uint8)).to(dev)  # noqa: E731
    cwk = d.gen_batch_device(r(K, nb), r(K, lam), r(K, lam), r(K, lam), dcf.BoundState.GtBeta)
    assert d.eval_multikey_device(True, cwk, r(K, lam), e(0, nb), 0).shape == (0, lam)
    torch.cuda.synchronize()
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    xs = _rand(rng, (70, nb))
    xs[0] = np.frombuffer(alpha, np.uint8)
    got = d.eval(False, dcf.Share([s0], k.cws, k.cw_np1), xs)
    assert np.array_equal(got, O.eval_(P, 0, ok, s0, xs, nthreads=8))


@pytest.mark.parametrize("nb,m", [(16, 3000), (4, 70_000), (16, 100_000), (2, 1000)])
def test_host_mid_path_vs_device_and_oracle(dcf, nb, m):
    """Auto mode, host buffers, a batch in the small-batch kernels' range: dcf_eval reads x from and
    writes y to a mapped pinned buffer (no staging DMAs).  Both parties: equal to the device-resident
    eval of the same points and, on a sample (every row at m <= 3000), to the oracle."""
    import torch
    rng = np.random.default_rng(0x1D + nb + m)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf.share_to_cwb(k, nb, 16), np.uint8).copy()).cuda()
    xs = _rand(rng, (m, nb))
    xs[0] = np.frombuffer(alpha, np.uint8)
    idx = np.arange(m) if m <= 3000 else np.concatenate([np.arange(1500), np.arange(m - 1500, m)])
    for b, s in ((0, s0), (1, s1)):
        got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
        dev = d.eval_device(bool(b), cwb, torch.from_numpy(np.frombuffer(s, np.uint8).copy()).cuda(),
                            torch.from_numpy(xs).cuda())
        torch.cuda.synchronize()
        assert np.array_equal(got, dev.cpu().numpy()), b
        assert np.array_equal(got[idx], O.eval_(P, b, ok, s, xs[idx], nthreads=8)), b
    # the same buffer refilled with other points right away (the kernel must not see the
    # previous call's x through a cached line)
    for rep in range(3):
        xs2 = _rand(rng, (m, nb))
        got2 = d.eval(False, dcf.Share([s0], k.cws, k.cw_np1), xs2)
        dev2 = d.eval_device(False, cwb, torch.from_numpy(np.frombuffer(s0, np.uint8).copy()).cuda(),
                             torch.from_numpy(xs2).cuda())
        torch.cuda.synchronize()
        assert np.array_equal(got2, dev2.cpu().numpy()), rep
