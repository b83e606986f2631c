"""Aes128MatyasMeyerOseasPrg (BASELINE.json north_star).

The reference crate has no MMO PRG, so this PRG's definition is ours
(include/dcf_hip.h, dcf_mmo_prg_new) and its parity is UNPINNED by the
reference.  What pins it: AES-128 against FIPS-197 C.1 and libcrypto; the C
oracle against the independent Python/libcrypto restatement (the committed
fixtures tests/golden/mmo16.json, written only when both agree); the DCF
reconstruction property y0 ^ y1 = beta * [x < alpha] (lib.rs:372-420's check);
and, on the GPU, the HIP kernels bit for bit against the oracle.
"""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import pyref as R
from tests.golden.make_golden import detbytes


def _keys(g):
    return [bytes.fromhex(k) for k in g["keys"]]


def test_aes128_fips197_and_kat(golden):
    for v in golden("mmo16")["aes128_kat"]:
        assert O.aes128_encrypt(bytes.fromhex(v["key"]), bytes.fromhex(v["pt"])).hex() == v["ct"]


@pytest.mark.parametrize("aesni", [True, False])
def test_mmo_prg_golden(golden, aesni):
    g = golden("mmo16")
    P = O.OracleMmoPrg(_keys(g), 16, allow_aesni=aesni)
    for r in g["prg_rows"]:
        (sl, vl, tl), (sr, vr, tr) = P.gen(bytes.fromhex(r["seed"]))
        assert (sl.hex(), vl.hex(), tl, sr.hex(), vr.hex(), tr) == (r["sl"], r["vl"], r["tl"], r["sr"], r["vr"],
                                                                      r["tr"])


def test_mmo_prg_definition():
    """The definition itself, restated inline: blockwise E_k(m) ^ m, t from byte 0 bit 0 of
    s_L / s_R before the clear, last byte's bit 0 cleared."""
    keys = [detbytes(f"mmo/def/{i}", 16) for i in range(8)]
    P = O.OracleMmoPrg(keys, 32)
    seed = detbytes("mmo/def/seed", 32)
    outs = []
    for b in range(4):
        o = bytearray()
        for j in range(2):
            blk = seed[16 * j:16 * j + 16]
            o += bytes(x ^ y for x, y in zip(O.aes128_encrypt(keys[2 * b + j], blk), blk))
        outs.append(o)
    t = (bool(outs[0][0] & 1), bool(outs[2][0] & 1))
    for o in outs:
        o[31] &= 0xFE
    assert P.gen(seed) == [(bytes(outs[0]), bytes(outs[1]), t[0]), (bytes(outs[2]), bytes(outs[3]), t[1])]


def test_mmo_cipher_n_too_small_rejected():
    with pytest.raises(ValueError):
        O.OracleMmoPrg([bytes(16)] * 3, 16)
    with pytest.raises(ValueError):
        O.OracleMmoPrg([bytes(16)] * 7, 32)


def test_mmo_dcf_golden_cases(golden):
    g = golden("mmo16")
    P = O.OracleMmoPrg(_keys(g), 16)
    for c in g["cases"]:
        nb = c["n_bytes"]
        s0s = [bytes.fromhex(s) for s in c["s0s"]]
        k = O.gen(P, bytes.fromhex(c["alpha"]), bytes.fromhex(c["beta"]), s0s[0], s0s[1], c["bound"])
        raw = k.cw_s.tobytes() + k.cw_v.tobytes() + k.cw_t.tobytes()
        assert (raw + bytes((-len(raw)) % 16) + k.cw_np1.tobytes()).hex() == c["cwb"], c["name"]
        xs = np.array([list(bytes.fromhex(x)) for x in c["xs"]], np.uint8).reshape(-1, nb)
        for b, key in ((0, "y0"), (1, "y1")):
            ys = O.eval_(P, b, k, s0s[b], xs)
            assert [y.tobytes().hex() for y in ys] == c[key], (c["name"], b)


@pytest.mark.parametrize("bound", [0, 1])
def test_mmo_reconstruction_full_domain_cpu(bound):
    keys = [detbytes(f"mmo/rec/{i}", 16) for i in range(4)]
    P, Q = O.OracleMmoPrg(keys, 16), R.MmoPrg(keys, 16)
    alpha, beta = detbytes(f"mmo/rec/alpha/{bound}", 2), detbytes("mmo/rec/beta", 16)
    s0, s1 = detbytes("mmo/rec/s0", 16), detbytes("mmo/rec/s1", 16)
    k = O.gen(P, alpha, beta, s0, s1, bound)
    cws, np1 = R.gen(Q, alpha, beta, [s0, s1], bound)
    assert np1 == k.cw_np1.tobytes()
    xs = np.array([list(i.to_bytes(2, "big")) for i in range(1 << 16)], np.uint8)
    rec = O.eval_(P, 0, k, s0, xs, 8) ^ O.eval_(P, 1, k, s1, xs, 8)
    a = int.from_bytes(alpha, "big")
    hit = np.arange(1 << 16) < a if bound == 0 else np.arange(1 << 16) > a
    assert (rec[hit] == np.frombuffer(beta, np.uint8)).all() and not rec[~hit].any()


# ---------------- GPU: the HIP kernels against the oracle ----------------

@pytest.fixture(scope="module")
def dcf(hip_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import dcf_amd
    return dcf_amd


@pytest.mark.gpu
def test_gpu_mmo_prg_golden(dcf, golden):
    g = golden("mmo16")
    prg = dcf.Aes128MatyasMeyerOseasPrg(_keys(g), 16)
    assert dcf.load().dcf_prg_kind(prg.handle) == 1
    outs = prg.gen_many([bytes.fromhex(r["seed"]) for r in g["prg_rows"]])
    for r, ((sl, vl, tl), (sr, vr, tr)) in zip(g["prg_rows"], outs):
        assert (sl.hex(), vl.hex(), tl, sr.hex(), vr.hex(), tr) == (r["sl"], r["vl"], r["tl"], r["sr"], r["vr"],
                                                                      r["tr"])


@pytest.mark.gpu
def test_gpu_mmo_gen_eval_golden(dcf, golden):
    g = golden("mmo16")
    prg = dcf.Aes128MatyasMeyerOseasPrg(_keys(g), 16)
    for c in g["cases"]:
        nb = c["n_bytes"]
        d = dcf.DcfImpl(nb, 16, prg)
        s0s = [bytes.fromhex(s) for s in c["s0s"]]
        k = d.gen(dcf.CmpFn(bytes.fromhex(c["alpha"]), bytes.fromhex(c["beta"])), s0s, dcf.BoundState(c["bound"]))
        assert dcf.share_to_cwb(k, nb, 16).hex() == c["cwb"], c["name"]
        xs = [bytes.fromhex(x) for x in c["xs"]]
        for b, key in ((0, "y0"), (1, "y1")):
            ys = d.eval(bool(b), dcf.Share([s0s[b]], k.cws, k.cw_np1), xs)
            assert [y.tobytes().hex() for y in ys] == c[key], (c["name"], b)


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [1, 2, 4, 5, 16, 17])
def test_gpu_mmo_eval_random_vs_oracle(dcf, nb):
    rng = np.random.default_rng(700 + nb)
    keys = [rng.bytes(16) for _ in range(4)]
    prg, P = dcf.Aes128MatyasMeyerOseasPrg(keys, 16), O.OracleMmoPrg(keys, 16)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    ok = O.gen(P, alpha, beta, s0, s1, nb % 2)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(nb % 2))
    raw = ok.cw_s.tobytes() + ok.cw_v.tobytes() + ok.cw_t.tobytes()
    assert dcf.share_to_cwb(k, nb, 16) == raw + bytes((-len(raw)) % 16) + ok.cw_np1.tobytes()
    for m in (0, 1, 63, 65, 777):
        xs = rng.integers(0, 256, size=(m, nb), dtype=np.uint8)
        if m > 3:
            xs[0] = np.frombuffer(alpha, np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=4)), (nb, m, b)


@pytest.mark.gpu
@pytest.mark.parametrize("K,P", [(37, 64), (10, 13)])
def test_gpu_mmo_batch_gen_multikey_eval(dcf, K, P):
    import torch
    nb = 16
    rng = np.random.default_rng(K * 31 + P)
    keys = [rng.bytes(16) for _ in range(4)]
    prg, Po = dcf.Aes128MatyasMeyerOseasPrg(keys, 16), O.OracleMmoPrg(keys, 16)
    d = dcf.DcfImpl(nb, 16, prg)
    r = lambda *s: rng.integers(0, 256, size=s, dtype=np.uint8)  # noqa: E731
    alpha, beta, s0, s1 = r(K, nb), r(K, 16), r(K, 16), r(K, 16)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf.BoundState.LtBeta)
    xs = r(K * P, nb)
    y0 = d.eval_multikey_device(False, cwb, T(s0), T(xs), P)
    y1 = d.eval_multikey_device(True, cwb, T(s1), T(xs), P)
    torch.cuda.synchronize()
    cw, y0h, y1h = cwb.cpu().numpy(), y0.cpu().numpy(), y1.cpu().numpy()
    n = 8 * nb
    cws = cw[:n * K * 16].reshape(n, K, 16)
    for key in sorted({0, K - 1, K // 2}):
        ok = O.gen(Po, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), 0)
        assert np.array_equal(cws[:, key], ok.cw_s)
        sl = slice(key * P, (key + 1) * P)
        assert np.array_equal(y0h[sl], O.eval_(Po, 0, ok, s0[key].tobytes(), xs[sl]))
        assert np.array_equal(y1h[sl], O.eval_(Po, 1, ok, s1[key].tobytes(), xs[sl]))


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [1, 2])
def test_gpu_mmo_full_domain(dcf, nb):
    import torch
    rng = np.random.default_rng(900 + nb)
    keys = [rng.bytes(16) for _ in range(4)]
    prg, P = dcf.Aes128MatyasMeyerOseasPrg(keys, 16), O.OracleMmoPrg(keys, 16)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    cwb = torch.from_numpy(np.frombuffer(dcf.share_to_cwb(k, nb, 16), np.uint8).copy()).cuda()
    xs = np.array([list(i.to_bytes(nb, "big")) for i in range(1 << (8 * nb))], np.uint8)
    for b, s in ((0, s0), (1, s1)):
        y = d.eval_full_domain_device(bool(b), cwb, torch.from_numpy(np.frombuffer(s, np.uint8).copy()).cuda())
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy(), O.eval_(P, b, ok, s, xs, nthreads=8)), (nb, b)


@pytest.mark.gpu
def test_gpu_mmo_errors(dcf):
    with pytest.raises(dcf.DcfError) as e:
        dcf.Aes128MatyasMeyerOseasPrg([bytes(16)] * 3, 16)
    assert e.value.code == -3
    with pytest.raises(dcf.DcfError) as e:
        dcf.Aes128MatyasMeyerOseasPrg([bytes(16)] * 7, 32)  # LAMBDA = 32 needs 4 * 2 keys
    assert e.value.code == -3
    prg = dcf.Aes128MatyasMeyerOseasPrg([bytes(16)] * 8, 32)  # multi-block MMO is supported
    assert prg.eval_prefix_levels(2, 1, 1 << 20) == 0        # no shared prefix at LAMBDA >= 32


def _mmo_keys(lam, seed):
    rng = np.random.default_rng(seed)
    return rng, [rng.bytes(16) for _ in range(4 * lam // 16)]


@pytest.mark.gpu
@pytest.mark.parametrize("lam", [32, 48, 64, 256, 16384])
def test_gpu_mmo_wide_prg_vs_oracle(dcf, lam):
    """Multi-block MMO (one AES-128 key per output and 16-byte block) on the GPU PRG hook
    vs the oracle's definition (checked against the inline restatement above)."""
    rng, keys = _mmo_keys(lam, lam)
    prg, P = dcf.Aes128MatyasMeyerOseasPrg(keys, lam), O.OracleMmoPrg(keys, lam)
    seeds = [rng.bytes(lam) for _ in range(7)]
    assert prg.gen_many(seeds) == [P.gen(sd) for sd in seeds]


@pytest.mark.gpu
@pytest.mark.parametrize("lam,nb,m", [(32, 2, 300), (48, 3, 200), (64, 16, 130), (512, 4, 100), (16384, 16, 70),
                                      (32, 1, 256), (96, 5, 65), (64, 31, 70), (48, 32, 70), (64, 40, 65),
                                      (32, 100, 40)])
def test_gpu_mmo_wide_gen_eval_vs_oracle(dcf, lam, nb, m):
    """gen + eval of both parties and both bounds at LAMBDA >= 32 (head over block 0, tail over
    the others) bit for bit with the oracle, and the reconstruction y0 ^ y1 = beta [x < alpha]
    (LtBeta) / [x > alpha] (GtBeta) on every point (parity unpinned by the reference).  N >= 32:
    the t-vector passes 8 words (t_0 .. t_n, n + 1 > 256 bits)."""
    rng, keys = _mmo_keys(lam, lam * 3 + nb)
    prg, P = dcf.Aes128MatyasMeyerOseasPrg(keys, lam), O.OracleMmoPrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    for bound in (0, 1):
        alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        raw = ok.cw_s.tobytes() + ok.cw_v.tobytes() + ok.cw_t.tobytes()
        assert dcf.share_to_cwb(k, nb, lam) == raw + bytes((-len(raw)) % 16) + ok.cw_np1.tobytes(), (lam, bound)
        xs = rng.integers(0, 256, (m, nb), dtype=np.uint8)
        xs[0] = np.frombuffer(alpha, np.uint8)
        ys = []
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), (lam, nb, bound, b)
            ys.append(got)
        xi = [int.from_bytes(x.tobytes(), "big") for x in xs]
        a = int.from_bytes(alpha, "big")
        for i, x in enumerate(xi):
            on = (x < a) if bound == 0 else (x > a)
            assert (ys[0][i] ^ ys[1][i]).tobytes() == (beta if on else bytes(lam)), (i, bound)


@pytest.mark.gpu
def test_gpu_mmo_wide_batch_gen_multikey_and_full_domain(dcf):
    """Batched gen (64-key waves, a ragged last wave) + multi-key eval at LAMBDA = 64, and the
    full-domain eval at N = 1, LAMBDA = 32, against the oracle."""
    import torch
    lam, nb, K, Pp = 64, 2, 70, 9
    rng, keys = _mmo_keys(lam, 4242)
    prg, Po = dcf.Aes128MatyasMeyerOseasPrg(keys, lam), O.OracleMmoPrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    r = lambda *sh: rng.integers(0, 256, sh, dtype=np.uint8)  # noqa: E731
    alpha, beta, s0, s1 = r(K, nb), r(K, lam), r(K, lam), r(K, lam)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf.BoundState.GtBeta)
    xs = r(K * Pp, nb)
    y0 = d.eval_multikey_device(False, cwb, T(s0), T(xs), Pp)
    torch.cuda.synchronize()
    cw, y0h = cwb.cpu().numpy(), y0.cpu().numpy()
    n = 8 * nb
    cws = cw[:n * K * lam].reshape(n, K, lam)
    for key in (0, 1, 63, 64, K - 1):
        ok = O.gen(Po, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), 1)
        assert np.array_equal(cws[:, key], ok.cw_s), key
        sl = slice(key * Pp, (key + 1) * Pp)
        assert np.array_equal(y0h[sl], O.eval_(Po, 0, ok, s0[key].tobytes(), xs[sl])), key
    lam, nb = 32, 1
    rng, keys = _mmo_keys(lam, 99)
    prg, Po = dcf.Aes128MatyasMeyerOseasPrg(keys, lam), O.OracleMmoPrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    ok = O.gen(Po, alpha, beta, s0, s1, 0)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    cwbt = torch.from_numpy(np.frombuffer(dcf.share_to_cwb(k, nb, lam), np.uint8).copy()).cuda()
    y = d.eval_full_domain_device(False, cwbt, torch.from_numpy(np.frombuffer(s0, np.uint8).copy()).cuda())
    torch.cuda.synchronize()
    xs = np.arange(256, dtype=np.uint8).reshape(256, 1)
    assert np.array_equal(y.cpu().numpy(), O.eval_(Po, 0, ok, s0, xs))


@pytest.mark.gpu
@pytest.mark.parametrize("nb,levels", [(1, 1), (1, 7), (2, 15), (3, 23), (4, 24), (16, 13), (16, 24), (17, 20)])
def test_gpu_mmo_eval_prefix_table_vs_oracle(dcf, nb, levels):
    """Shared-prefix eval with the MMO PRG (forced depth D): points start at level D
    from the key's top tree, expanded by the MMO full-domain level kernel; output
    unchanged.  D = 8N - 1, D across x's word boundary and the 24-level cap."""
    rng = np.random.default_rng(900 + 31 * nb + levels)
    keys = [rng.bytes(16) for _ in range(4)]
    prg, P = dcf.Aes128MatyasMeyerOseasPrg(keys, 16), O.OracleMmoPrg(keys, 16)
    prg.set_prefix_levels(levels)
    m = 3001
    assert prg.eval_prefix_levels(nb, 1, m) == min(levels, 24, 8 * nb - 1)
    d = dcf.DcfImpl(nb, 16, prg)
    for bound in (0, 1):
        alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
        ok = O.gen(P, alpha, beta, s0, s1, bound)
        k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
        xs = rng.integers(0, 256, size=(m, nb), dtype=np.uint8)
        a = np.frombuffer(alpha, np.uint8)
        xs[0], xs[1], xs[2] = a, 0, 255
        xs[3:40] = a
        xs[3:40, -1] = rng.integers(0, 256, 37, dtype=np.uint8)
        for b, s in ((0, s0), (1, s1)):
            got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
            assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), (nb, levels, bound, b)
    prg.set_prefix_levels(-1)
    assert prg.eval_prefix_levels(16, 1, m) == 0           # auto: no table for small batches
    assert prg.eval_prefix_levels(16, 1, 1 << 22) == 21    # auto: log2(points) - 1
    assert prg.eval_prefix_levels(16, 2, 1 << 22) == 0     # one key only
