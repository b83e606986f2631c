"""Seeded random-shape parity sweep (GPU): many (N, LAMBDA, PRG, bound, batch) combinations
that the hand-picked parity cases do not name, each checked bit for bit against the C oracle
(oracle/dcf_oracle.c: lib.rs:86-204 over prg.rs:42-73, or the MMO PRG of include/dcf_hip.h).

Every case runs gen through the C ABI and compares the CWB with the oracle's key
(lib.rs:86-161), then evaluates both parties (lib.rs:163-204) on random points with x = alpha
planted (host-buffer entry point; batches of 64 or more also through the device-buffer one),
and checks y0 ^ y1 against beta * [x < alpha] / [x > alpha] (lib.rs:114-125 and the
reconstruction KATs, lib.rs:372-420).  The shapes come from a fixed seed, so a failure names a
reproducible case id.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

LAMS = [16, 16, 16, 32, 48, 64, 80, 96, 112, 128, 144, 256, 272, 384, 512, 1024]


# Extended sweeps (one-off GPU runs; the default is the suite's fixed list): DCF_FUZZ_CASES /
# DCF_FUZZ_MK_CASES cases from DCF_FUZZ_SEED / DCF_FUZZ_MK_SEED, and with DCF_FUZZ_BIG=1 also
# λ = 16 batches on the pair-walk (40000 points) and stream (600000) engines.
_ENV = os.environ.get


def _cases(n=int(_ENV("DCF_FUZZ_CASES", "128")), seed=int(_ENV("DCF_FUZZ_SEED", "0xF022"), 0)):
    rng = np.random.default_rng(seed)
    big = _ENV("DCF_FUZZ_BIG") == "1"
    out = []
    for i in range(n):
        lam = int(rng.choice(LAMS))
        nb = int(rng.integers(1, 41 if lam == 16 else 25))
        mmo = bool(rng.random() < 0.25)
        m = int(rng.choice([1, 2, 17, 64, 65, 300, 1000, 2049, 4097]))
        if lam >= 512:
            m = min(m, 300)
        if big and lam == 16 and rng.random() < 0.3:
            m = int(rng.choice([40000, 600000]))
        out.append((i, lam, nb, mmo, int(rng.integers(0, 2)), m))
    return out


def _mk_cases(n=int(_ENV("DCF_FUZZ_MK_CASES", "24")), seed=int(_ENV("DCF_FUZZ_MK_SEED", "0xF0A2"), 0)):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        lam = int(rng.choice([16, 16, 32, 64, 128, 256]))
        nb = int(rng.integers(1, 21))
        K = int(rng.integers(1, 300))
        P = int(rng.choice([1, 5, 31, 32, 33, 64, 100]))
        out.append((i, lam, nb, K, P))
    return out


def _prgs(dcf, rng, lam, mmo):
    if mmo:
        keys = [rng.bytes(16) for _ in range(max(4, 4 * lam // 16))]
        return dcf.Aes128MatyasMeyerOseasPrg(keys, lam), O.OracleMmoPrg(keys, lam)
    keys = [rng.bytes(32) for _ in range(18 if lam > 16 else 2)]
    return dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)


def _cwb_of(ok, lam):
    raw = ok.cw_s.tobytes() + ok.cw_v.tobytes() + ok.cw_t.tobytes()
    return raw + bytes((-len(raw)) % 16) + ok.cw_np1.tobytes()


def _lt(xs, a):
    """[x < alpha] per row (big-endian, Msb0 as lib.rs:181)."""
    diff = xs != a
    has = diff.any(1)
    first = diff.argmax(1)
    r = np.arange(xs.shape[0])
    return has & (xs[r, first] < a[first])


@pytest.fixture(scope="module")
def dcf(hip_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import dcf_amd
    return dcf_amd


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"c{c[0]}-lam{c[1]}-n{c[2]}-{'mmo' if c[3] else 'hirose'}-b{c[4]}-m{c[5]}")
def test_fuzz_single_key_vs_oracle(dcf, case):
    i, lam, nb, mmo, bound, m = case
    rng = np.random.default_rng(0x5EED + i)
    prg, P = _prgs(dcf, rng, lam, mmo)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    ok = O.gen(P, alpha, beta, s0, s1, bound)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
    assert dcf.share_to_cwb(k, nb, lam) == _cwb_of(ok, lam), "gen differs from the oracle"
    xs = rng.integers(0, 256, size=(m, nb), dtype=np.uint8)
    a = np.frombuffer(alpha, np.uint8)
    xs[0] = a
    if m > 8:  # neighbours of alpha: equal prefix, last byte on either side
        xs[1:8] = a
        xs[1:8, -1] = (a[-1] + np.array([1, 255, 2, 254, 128, 3, 253], np.uint8)) & 0xFF
    ys = []
    for b, s in ((0, s0), (1, s1)):
        got = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
        assert np.array_equal(got, O.eval_(P, b, ok, s, xs, nthreads=8)), f"party {b}"
        ys.append(np.asarray(got))
    if m >= 64:  # the device-buffer entry point gives the same bytes
        import torch
        T = lambda v: torch.from_numpy(np.frombuffer(v, np.uint8).copy() if isinstance(v, bytes) else v).cuda()  # noqa: E731
        yd = d.eval_device(True, T(dcf.share_to_cwb(k, nb, lam)), T(s1), T(xs))
        torch.cuda.synchronize()
        assert np.array_equal(yd.cpu().numpy(), ys[1]), "eval_device"
    if bound == 0:
        want = np.where(_lt(xs, a)[:, None], np.frombuffer(beta, np.uint8)[None, :], 0)
    else:  # GtBeta: beta where x > alpha
        gt = (~_lt(xs, a)) & (xs != a).any(1)
        want = np.where(gt[:, None], np.frombuffer(beta, np.uint8)[None, :], 0)
    assert np.array_equal(ys[0] ^ ys[1], want.astype(np.uint8)), "reconstruction"


@pytest.mark.parametrize("case", _mk_cases(), ids=lambda c: f"k{c[0]}-lam{c[1]}-n{c[2]}-K{c[3]}-P{c[4]}")
def test_fuzz_multikey_vs_oracle(dcf, case):
    """Batched gen of K keys and multi-key eval of P points per key (every engine the shape
    selects: per-key top trees, batched λ ≥ 32 passes, the root-seed start path)."""
    import torch
    i, lam, nb, K, P = case
    rng = np.random.default_rng(0x3EED + i)
    prg, Po = _prgs(dcf, rng, lam, False)
    d = dcf.DcfImpl(nb, lam, prg)
    r = lambda *s: rng.integers(0, 256, size=s, dtype=np.uint8)  # noqa: E731
    alpha, beta, s0, s1 = r(K, nb), r(K, lam), r(K, lam), r(K, lam)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    cwb = d.gen_batch_device(T(alpha), T(beta), T(s0), T(s1), dcf.BoundState.LtBeta)
    xs = r(K * P, nb)
    xs[::P] = alpha
    y0 = d.eval_multikey_device(False, cwb, T(s0), T(xs), P)
    y1 = d.eval_multikey_device(True, cwb, T(s1), T(xs), P)
    torch.cuda.synchronize()
    y0h, y1h = y0.cpu().numpy(), y1.cpu().numpy()
    for key in sorted({0, K - 1, int(rng.integers(0, K))}):
        ok = O.gen(Po, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), 0)
        sl = slice(key * P, (key + 1) * P)
        assert np.array_equal(y0h[sl], O.eval_(Po, 0, ok, s0[key].tobytes(), xs[sl], nthreads=8)), key
        assert np.array_equal(y1h[sl], O.eval_(Po, 1, ok, s1[key].tobytes(), xs[sl], nthreads=8)), key
    lt = np.stack([_lt(xs[k * P:(k + 1) * P], alpha[k]) for k in range(K)])
    want = np.where(lt.reshape(-1)[:, None], np.repeat(beta, P, 0), 0).astype(np.uint8)
    assert np.array_equal(y0h ^ y1h, want), "reconstruction"
