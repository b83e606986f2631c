"""Full-size parity for every BASELINE.json config.

Each test runs the config at its real size on the MI355X through the C ABI and
checks it two ways:
  * bit-exact against the CPU oracle (oracle/dcf_oracle.c, the restatement of
    lib.rs:163-204 + prg.rs:42-73) on a sample of >= 8k points that includes the
    first and last points of every work unit / pass boundary the kernels use;
  * the reconstruction property of the reference's own tests (lib.rs:372-420),
    y0 ^ y1 == beta * [x < alpha] (LtBeta), on EVERY point, vectorised on the GPU.
Shapes: benches/dcf_batch_eval.rs:17-33 (C1) and benches/dcf_large_lambda.rs:8-21
(C4), scaled as BASELINE.json states.  These run after the rest of the GPU suite
(tests/conftest.py orders them last) and take ~1-2 min together.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.config]

CPU_THREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def dcf(hip_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import dcf_amd
    return dcf_amd


def oracle_key(dcf, cwb: bytes, nb: int, lam: int, K: int = 1, key: int = 0) -> "O.OracleKey":
    """Key `key` of a K-key CWB (include/dcf_hip.h layout) as an oracle key."""
    n = 8 * nb
    c = np.frombuffer(cwb, np.uint8)
    k = O.OracleKey(nb, lam)
    k.cw_s[:] = c[:n * K * lam].reshape(n, K, lam)[:, key]
    k.cw_v[:] = c[n * K * lam:2 * n * K * lam].reshape(n, K, lam)[:, key]
    k.cw_t[:] = c[2 * n * K * lam:2 * n * K * lam + n * K].reshape(n, K)[:, key]
    off = dcf.cwb_np1_offset(nb, lam, K)
    k.cw_np1[:] = c[off:off + K * lam].reshape(K, lam)[key]
    return k


def sample_index(m: int, unit: int, rng, extra: int = 8192):
    """First/last 4096 points, the first and last point of every `unit`-point work
    unit (stream refills, tail workgroups, passes), and `extra` random points."""
    starts = np.arange(0, m, unit)
    ends = np.minimum(starts + unit, m) - 1
    idx = np.concatenate([np.arange(min(m, 4096)), np.arange(max(0, m - 4096), m), starts, ends,
                          rng.integers(0, m, extra)])
    return np.unique(idx)


def lt_mask(xs, alpha):
    """[x < alpha] for every row of xs (big-endian bytes, Msb0 as lib.rs:181), on device.
    alpha: (N,) or (m, N) uint8 tensor."""
    import torch
    a = alpha.expand_as(xs) if alpha.dim() == 1 else alpha
    diff = xs != a
    has = diff.any(1)
    first = diff.to(torch.uint8).argmax(1, keepdim=True)
    return has & (xs.gather(1, first) < a.gather(1, first)).squeeze(1)


def check_reconstruction(xs, alpha, beta, y0, y1, chunk: int = 1 << 24):
    """y0 ^ y1 == beta * [x < alpha] on every point (BoundState::LtBeta, lib.rs:114-125).
    alpha / beta: one key's (N,) / (LAMBDA,) or per-point (m, N) / (m, LAMBDA) tensors."""
    import torch
    m = xs.shape[0]
    for off in range(0, m, chunk):
        sl = slice(off, min(m, off + chunk))
        lt = lt_mask(xs[sl], alpha if alpha.dim() == 1 else alpha[sl])
        rec = y0[sl] ^ y1[sl]
        b = beta if beta.dim() == 1 else beta[sl]
        want = torch.where(lt.unsqueeze(1), b.expand_as(rec) if b.dim() == 1 else b, torch.zeros_like(rec))
        bad = (rec != want).any(1)
        assert not bool(bad.any()), f"reconstruction fails at point {off + int(bad.nonzero()[0, 0])}"


def check_sample(P, k, s0: bytes, party: int, xs_dev, ys_dev, idx):
    import torch
    ti = torch.from_numpy(idx).to(xs_dev.device)
    xs = xs_dev[ti].cpu().numpy()
    want = O.eval_(P, party, k, s0, xs, nthreads=CPU_THREADS)
    got = ys_dev[ti].cpu().numpy()
    bad = np.nonzero((got != want).any(1))[0]
    assert bad.size == 0, f"party {party}: {bad.size} of {idx.size} sampled points differ, first at {idx[bad[0]]}"


def single_key_setup(dcf, nb, lam, cipher_n, seed):
    import torch
    rng = np.random.default_rng(seed)
    keys = [rng.bytes(32) for _ in range(cipher_n)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    cwb = dcf.share_to_cwb(k, nb, lam)
    ok = O.gen(P, alpha, beta, s0, s1, 0)
    assert cwb == bytes(np.concatenate([ok.cw_s.ravel(), ok.cw_v.ravel(), ok.cw_t,
                                        np.zeros((-(ok.cw_s.size * 2 + ok.cw_t.size)) % 16, np.uint8),
                                        ok.cw_np1])), "gen differs from the oracle"
    T = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()  # noqa: E731
    return rng, prg, P, d, k, ok, (alpha, beta, s0, s1), T


def test_config_c1(dcf):
    """C1: benches/dcf_batch_eval.rs:7-33 — N = 16, LAMBDA = 16, Aes256HirosePrg with 2 AES
    keys, one LtBeta key, 100 000 random points, BOTH parties, auto engine; through the
    host-pointer entry point (what DcfHip::eval calls) and the device one.  All 100k
    points are checked against the oracle."""
    import torch
    nb, lam, m = 16, 16, 100_000
    rng, prg, P, d, k, ok, (alpha, beta, s0, s1), T = single_key_setup(dcf, nb, lam, 2, 0xC1)
    assert prg.eval_prefix_levels(nb, 1, m) == 18  # small batch, auto: a depth-18 table below the pair walk (r06)
    xs = rng.integers(0, 256, (m, nb), dtype=np.uint8)
    xs[0] = np.frombuffer(alpha, np.uint8)
    ys_h = []
    for b, s in ((0, s0), (1, s1)):
        y = d.eval(bool(b), dcf.Share([s], k.cws, k.cw_np1), xs)
        assert np.array_equal(y, O.eval_(P, b, ok, s, xs, nthreads=CPU_THREADS)), f"party {b}"
        yd = d.eval_device(bool(b), T(dcf.share_to_cwb(k, nb, lam)), T(s), torch.from_numpy(xs).cuda())
        torch.cuda.synchronize()
        assert np.array_equal(yd.cpu().numpy(), y), f"device path differs, party {b}"
        ys_h.append(torch.from_numpy(y).cuda())
    check_reconstruction(torch.from_numpy(xs).cuda(), T(alpha), T(beta), ys_h[0], ys_h[1])


def _single_key_device(dcf, nb, m, want_depth, seed, unit):
    import torch
    lam = 16
    rng, prg, P, d, k, ok, (alpha, beta, s0, s1), T = single_key_setup(dcf, nb, lam, 2, seed)
    assert prg.eval_prefix_levels(nb, 1, m) == want_depth
    cwb = T(dcf.share_to_cwb(k, nb, lam))
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    xs = torch.randint(0, 256, (m, nb), dtype=torch.uint8, device="cuda", generator=g)
    xs[0] = T(alpha)
    xs[1:64] = T(alpha)                   # alpha's whole prefix, last byte varied
    xs[1:64, -1] = torch.arange(63, dtype=torch.uint8, device="cuda") * 4
    xs[64] = 0
    xs[65] = 255
    y0 = d.eval_device(False, cwb, T(s0), xs)
    y1 = d.eval_device(True, cwb, T(s1), xs)
    torch.cuda.synchronize()
    idx = sample_index(m, unit, rng)
    assert idx.size >= 8192
    check_sample(P, ok, s0, 0, xs, y0, idx)
    check_sample(P, ok, s1, 1, xs, y1, idx)
    check_reconstruction(xs, T(alpha), T(beta), y0, y1)


def test_config_c2(dcf):
    """C2: N = 4 (32-bit x), LAMBDA = 16, one key at 2^24 points, auto shared prefix D = 24."""
    _single_key_device(dcf, 4, 1 << 24, 24, 0xC2, 256)


def test_config_c3(dcf):
    """C3: N = 16 (128-bit x), LAMBDA = 16, one key at 2^28 points on one GPU (the bench's
    N = 1 shape), auto shared prefix D = 27; the sample holds both ends of every one of the
    2^20 256-point stream units (~2.1 M oracle evals per party, ~0.5 s on 16 threads)."""
    _single_key_device(dcf, 16, 1 << 28, 27, 0xC3, 256)


def test_config_c3_strong_slices(dcf):
    """C3 sharded over G = 8 GPUs (strong scaling, bench.py's default): each GPU evaluates
    a contiguous 2^25-point slice of the 2^28 points (dcf_point_slice), with its own auto
    prefix depth (25 instead of 27).  The first and last slices, evaluated alone, must
    equal the same rows of the whole-batch eval byte for byte."""
    import torch
    nb, lam = 16, 16
    rng, prg, P, d, k, ok, (alpha, beta, s0, s1), T = single_key_setup(dcf, nb, lam, 2, 0xC33)
    cwb = T(dcf.share_to_cwb(k, nb, lam))
    total, G = 1 << 28, 8
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC33)
    xs = torch.randint(0, 256, (total, nb), dtype=torch.uint8, device="cuda", generator=g)
    whole = d.eval_device(False, cwb, T(s0), xs)
    for sl in (0, G - 1):
        start, cnt = dcf.point_slice(total, G, sl)
        assert cnt == 1 << 25 and prg.eval_prefix_levels(nb, 1, cnt) == 25
        part = d.eval_device(False, cwb, T(s0), xs[start:start + cnt])
        torch.cuda.synchronize()
        assert torch.equal(part, whole[start:start + cnt]), sl
    idx = sample_index(total, 1 << 20, rng, extra=2048)
    check_sample(P, ok, s0, 0, xs, whole, idx)


def test_config_c4(dcf):
    """C4: benches/dcf_large_lambda.rs:8-21 — N = 16, LAMBDA = 16384, Aes256HirosePrg with
    2048 AES keys (ciphers 0 and 17 used), LtBeta, 2^22 points per GPU: one 2^22-point
    head/tail pass (auto wide prefix D = 21), 64 GiB of outputs per party, both parties.
    Sample: first/last 2048 points, the ends of every 4096-point tail workgroup, 2k random."""
    import torch
    nb, lam, m = 16, 16384, 1 << 22
    rng, prg, P, d, k, ok, (alpha, beta, s0, s1), T = single_key_setup(dcf, nb, lam, 2048, 0xC4)
    assert prg.eval_prefix_levels(nb, 1, m) == 21
    cwb = T(dcf.share_to_cwb(k, nb, lam))
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC4)
    xs = torch.randint(0, 256, (m, nb), dtype=torch.uint8, device="cuda", generator=g)
    xs[0] = T(alpha)
    xs[1:32] = T(alpha)
    xs[1:32, -1] = torch.arange(31, dtype=torch.uint8, device="cuda") * 8
    y0 = d.eval_device(False, cwb, T(s0), xs)
    y1 = d.eval_device(True, cwb, T(s1), xs)
    torch.cuda.synchronize()
    starts = np.arange(0, m, 4096)
    idx = np.unique(np.concatenate([np.arange(2048), np.arange(m - 2048, m), starts, starts + 4095,
                                    rng.integers(0, m, 2200)]))
    assert idx.size >= 8192
    for part in np.array_split(idx, 4):  # 16 KiB outputs: bounded host copies
        check_sample(P, ok, s0, 0, xs, y0, part)
        check_sample(P, ok, s1, 1, xs, y1, part)
    check_reconstruction(xs, T(alpha), T(beta), y0, y1, chunk=1 << 15)


@pytest.mark.parametrize("nb", [16, 4])
def test_config_c5(dcf, nb):
    """C5: 2^20 independent keys x 64 points, N = 16 (and N = 4), LAMBDA = 16:
    batched gen (one launch), then multi-key eval of both parties.  Sample: the CWB of 130 keys
    (first, last, random) against the oracle's gen and all 64 points of each (8320 evals per
    party); reconstruction on all 2^26 points with each key's alpha / beta."""
    import torch
    lam, K, Pk = 16, 1 << 20, 64
    rng = np.random.default_rng(0xC5 + nb)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, Po = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC5)
    r = lambda *s: torch.randint(0, 256, s, dtype=torch.uint8, device="cuda", generator=g)  # noqa: E731
    alpha, beta, s0, s1, xs = r(K, nb), r(K, lam), r(K, lam), r(K, lam), r(K * Pk, nb)
    xs[::Pk] = alpha  # x == alpha at each key's first point
    cwb = d.gen_batch_device(alpha, beta, s0, s1, dcf.BoundState.LtBeta)
    y0 = d.eval_multikey_device(False, cwb, s0, xs, Pk)
    y1 = d.eval_multikey_device(True, cwb, s1, xs, Pk)
    torch.cuda.synchronize()
    cw = cwb.cpu().numpy().tobytes()
    A, B, S0, S1 = (t.cpu().numpy() for t in (alpha, beta, s0, s1))
    sel = np.unique(np.concatenate([[0, 1, K - 2, K - 1], rng.integers(0, K, 126)]))
    for key in sel:
        ok = O.gen(Po, A[key].tobytes(), B[key].tobytes(), S0[key].tobytes(), S1[key].tobytes(), 0)
        kk = oracle_key(dcf, cw, nb, lam, K, int(key))
        assert np.array_equal(kk.cw_s, ok.cw_s) and np.array_equal(kk.cw_v, ok.cw_v), key
        assert np.array_equal(kk.cw_t, ok.cw_t) and np.array_equal(kk.cw_np1, ok.cw_np1), key
        pts = np.arange(key * Pk, (key + 1) * Pk)
        check_sample(Po, ok, S0[key].tobytes(), 0, xs, y0, pts)
        check_sample(Po, ok, S1[key].tobytes(), 1, xs, y1, pts)
    check_reconstruction(xs, alpha.repeat_interleave(Pk, 0), beta.repeat_interleave(Pk, 0), y0, y1)
