"""SURVEY §8 f1 on the GPU: keys in the reference's wire format feed the HIP path.

A dealer running the reference serialises each party's `Share` with bincode 1.x
(`bincode::serialize`, serde struct-as-seq, lib.rs:217-340; Cargo.toml:44) and the
evaluator decodes it.  Here the keys come from the CPU oracle's gen (the restatement of
lib.rs:86-161), are encoded by `spec_bincode` below — written from the bincode 1.x spec
and the serde derive order of `Share` / `Cw` alone, sharing no code with the library's
encoder — decoded by the C ABI's `dcf_share_from_bincode`, and evaluated by
`dcf_eval_device` / `dcf_eval_multikey_device`; every output byte must equal the oracle's
eval of the same key.  The opposite direction: keys made by `dcf_gen_batch_device` and
`dcf_gen`, serialised by `dcf_share_to_bincode`, must equal the spec encoding of the
oracle's gen byte for byte.  Bincode bytes of the Rust crate itself cannot be produced
here (no Rust toolchain): "parity unpinned" beyond the spec, as tests/test_wire.py says.
"""
import ctypes
import struct

import numpy as np
import pytest

from dcf_amd._lib import check
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CPU_THREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def dcf(hip_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import dcf_amd
    return dcf_amd


def spec_bincode(ok: "O.OracleKey", s0s, lam: int) -> bytes:
    """bincode 1.x of `Share { s0s: Vec<[u8; L]>, cws: Vec<Cw>, cw_np1: [u8; L] }` with
    `Cw { s, v, tl, tr }` (lib.rs:208-214, 275-283): fields in declaration order, u64 LE
    length before every sequence (the crate serialises each [u8; L] as a seq of L,
    lib.rs:223-226, 291-294), bool as one byte."""
    q = lambda v: struct.pack("<Q", v)  # noqa: E731
    out = [q(len(s0s))]
    for s in s0s:
        out += [q(lam), bytes(s)]
    out.append(q(ok.cw_s.shape[0]))
    for i in range(ok.cw_s.shape[0]):
        t = int(ok.cw_t[i])
        out += [q(lam), ok.cw_s[i].tobytes(), q(lam), ok.cw_v[i].tobytes(), bytes([t & 1, (t >> 1) & 1])]
    out += [q(lam), ok.cw_np1.tobytes()]
    return b"".join(out)


def abi_decode(dcf, data: bytes, nb: int, lam: int):
    """dcf_share_from_bincode -> (single-key CWB bytes, [seeds])."""
    L = dcf.load()
    cwb = ctypes.create_string_buffer(dcf.cwb_bytes(nb, lam, 1))
    seeds = ctypes.create_string_buffer(2 * lam)
    ns = ctypes.c_size_t(0)
    check(L.dcf_share_from_bincode(nb, lam, data, len(data), cwb, seeds, 2, ctypes.byref(ns)))
    return cwb.raw, [seeds.raw[i * lam:(i + 1) * lam] for i in range(ns.value)]


def abi_encode(dcf, cwb: bytes, seeds, nb: int, lam: int) -> bytes:
    L = dcf.load()
    n = int(L.dcf_share_bincode_bytes(nb, lam, len(seeds)))
    out = ctypes.create_string_buffer(n)
    check(L.dcf_share_to_bincode(nb, lam, cwb, b"".join(seeds), len(seeds), out, n))
    return out.raw


def key_of(cwb: np.ndarray, nb: int, lam: int, K: int, key: int, np1_off: int) -> bytes:
    """Single-key CWB of key `key` of a K-key CWB (include/dcf_hip.h layout)."""
    n = 8 * nb
    s = cwb[:n * K * lam].reshape(n, K, lam)[:, key]
    v = cwb[n * K * lam:2 * n * K * lam].reshape(n, K, lam)[:, key]
    t = cwb[2 * n * K * lam:2 * n * K * lam + n * K].reshape(n, K)[:, key]
    np1 = cwb[np1_off:np1_off + K * lam].reshape(K, lam)[key]
    raw = s.tobytes() + v.tobytes() + t.tobytes()
    return raw + bytes((-len(raw)) % 16) + np1.tobytes()


def stack_keys(cwbs, nb: int, lam: int, np1_off_k: int) -> bytes:
    """K single-key CWBs -> one K-key CWB (structure of arrays across keys)."""
    n, K = 8 * nb, len(cwbs)
    a = [np.frombuffer(c, np.uint8) for c in cwbs]
    s = np.stack([c[:n * lam].reshape(n, lam) for c in a], 1)
    v = np.stack([c[n * lam:2 * n * lam].reshape(n, lam) for c in a], 1)
    t = np.stack([c[2 * n * lam:2 * n * lam + n] for c in a], 1)
    np1 = np.stack([c[-lam:] for c in a], 0)
    raw = s.tobytes() + v.tobytes() + t.tobytes()
    raw += bytes(np1_off_k - len(raw))
    return raw + np1.tobytes()


# (N, LAMBDA, AES keys, points): the C3 / C2 shapes at 2^20 points (auto shared prefix:
# the table path and the stream engine), and benches/dcf_large_lambda.rs's LAMBDA = 16384
# with 2048 AES keys (wide head + tail) at 512 points.
SHAPES = [(16, 16, 2, 1 << 20), (4, 16, 2, 1 << 20), (16, 16384, 2048, 512)]


@pytest.mark.parametrize("bound", [0, 1])
@pytest.mark.parametrize("nb,lam,cipher_n,m", SHAPES)
def test_bincode_share_evaluates_on_gpu(dcf, nb, lam, cipher_n, m, bound):
    """Oracle gen -> spec bincode per party -> dcf_share_from_bincode -> dcf_eval_device,
    both parties, every output byte against the oracle's eval, and y0 ^ y1 against
    beta * [x < alpha] (LtBeta) / [x > alpha] (GtBeta) on every point (lib.rs:372-420)."""
    import torch
    rng = np.random.default_rng(0xF1 + 7 * nb + lam + bound)
    keys = [rng.bytes(32) for _ in range(cipher_n)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    ok = O.gen(P, alpha, beta, s0, s1, bound)
    # the dealer's full share (both seeds) round-trips through the ABI unchanged
    full = spec_bincode(ok, [s0, s1], lam)
    cwb_full, seeds_full = abi_decode(dcf, full, nb, lam)
    assert seeds_full == [s0, s1]
    assert abi_encode(dcf, cwb_full, seeds_full, nb, lam) == full
    xs = rng.integers(0, 256, (m, nb), dtype=np.uint8)
    xs[0] = np.frombuffer(alpha, np.uint8)
    xs[1] = 0
    xs[2] = 255
    xs[3:35] = np.frombuffer(alpha, np.uint8)
    xs[3:35, -1] = np.arange(32, dtype=np.uint8) * 8  # around alpha in its last byte
    xs_d = torch.from_numpy(xs).cuda()
    ys = []
    for b, s in ((0, s0), (1, s1)):
        wire_b = spec_bincode(ok, [s], lam)  # party b's share: s0s trimmed (lib.rs:382-385)
        cwb, seeds = abi_decode(dcf, wire_b, nb, lam)
        assert cwb == cwb_full and seeds == [s]
        cwb_d = torch.frombuffer(bytearray(cwb), dtype=torch.uint8).cuda()
        s_d = torch.frombuffer(bytearray(seeds[0]), dtype=torch.uint8).cuda()
        y = d.eval_device(bool(b), cwb_d, s_d, xs_d)
        torch.cuda.synchronize()
        got = y.cpu().numpy()
        want = O.eval_(P, b, ok, s, xs, nthreads=CPU_THREADS)
        bad = np.nonzero((got != want).any(1))[0]
        assert bad.size == 0, f"party {b}: {bad.size} of {m} points differ, first at {bad[:4]}"
        ys.append(got)
    rec = ys[0] ^ ys[1]
    xa = np.frombuffer(alpha, np.uint8)
    # big-endian compare (Msb0, lib.rs:181): first differing byte decides
    diff = xs != xa
    first = diff.argmax(1)
    rows = np.arange(m)
    lt = diff.any(1) & (xs[rows, first] < xa[first])
    gt = diff.any(1) & (xs[rows, first] > xa[first])
    hit = lt if bound == 0 else gt
    want_rec = np.where(hit[:, None], np.frombuffer(beta, np.uint8)[None, :], 0).astype(np.uint8)
    assert np.array_equal(rec, want_rec)


@pytest.mark.parametrize("nb,lam,cipher_n,K", [(16, 16, 2, 37), (4, 16, 2, 5), (16, 16384, 2048, 2)])
def test_gpu_gen_serialises_to_spec(dcf, nb, lam, cipher_n, K):
    """dcf_gen_batch_device keys (and one dcf_gen key) -> dcf_share_to_bincode == the spec
    encoding of the oracle's gen of the same (alpha, beta, seeds), both bounds."""
    import torch
    from dcf_amd import wire
    rng = np.random.default_rng(0xF1F + nb + lam + K)
    keys = [rng.bytes(32) for _ in range(cipher_n)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    r = lambda *s: rng.integers(0, 256, s, dtype=np.uint8)  # noqa: E731
    A, B, S0, S1 = r(K, nb), r(K, lam), r(K, lam), r(K, lam)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    for bound in (0, 1):
        cwb = d.gen_batch_device(T(A), T(B), T(S0), T(S1), dcf.BoundState(bound))
        torch.cuda.synchronize()
        c = cwb.cpu().numpy()
        off = dcf.cwb_np1_offset(nb, lam, K)
        for key in range(K):
            ok = O.gen(P, A[key].tobytes(), B[key].tobytes(), S0[key].tobytes(), S1[key].tobytes(), bound)
            seeds = [S0[key].tobytes(), S1[key].tobytes()]
            one = key_of(c, nb, lam, K, key, off)
            assert abi_encode(dcf, one, seeds, nb, lam) == spec_bincode(ok, seeds, lam), (bound, key)
            assert abi_encode(dcf, one, seeds[1:], nb, lam) == spec_bincode(ok, seeds[1:], lam), (bound, key)
        # the host entry point (what DcfHip::gen calls) serialises the same way
        k = d.gen(dcf.CmpFn(A[0].tobytes(), B[0].tobytes()), [S0[0].tobytes(), S1[0].tobytes()],
                  dcf.BoundState(bound))
        ok = O.gen(P, A[0].tobytes(), B[0].tobytes(), S0[0].tobytes(), S1[0].tobytes(), bound)
        assert wire.share_to_bincode(k, nb, lam) == spec_bincode(ok, k.s0s, lam)


def test_bincode_keys_batch_eval_on_gpu(dcf):
    """Many reference-format keys -> one multi-key launch (the C5 gate shape, scaled down):
    64 oracle keys, each party's share spec-encoded and decoded one by one, stacked into a
    64-key CWB, 64 points per key through dcf_eval_multikey_device, every byte against the
    oracle."""
    import torch
    nb, lam, K, Pk = 16, 16, 64, 64
    rng = np.random.default_rng(0xF15)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, lam), O.OraclePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    r = lambda *s: rng.integers(0, 256, s, dtype=np.uint8)  # noqa: E731
    A, B, S0, S1, xs = r(K, nb), r(K, lam), r(K, lam), r(K, lam), r(K * Pk, nb)
    xs[::Pk] = A
    oks = [O.gen(P, A[k].tobytes(), B[k].tobytes(), S0[k].tobytes(), S1[k].tobytes(), k % 2) for k in range(K)]
    off = dcf.cwb_np1_offset(nb, lam, K)
    for b, S in ((0, S0), (1, S1)):
        dec = [abi_decode(dcf, spec_bincode(oks[k], [S[k].tobytes()], lam), nb, lam) for k in range(K)]
        cwb = stack_keys([c for c, _ in dec], nb, lam, off)
        assert len(cwb) == dcf.cwb_bytes(nb, lam, K)
        s0s = np.frombuffer(b"".join(s[0] for _, s in dec), np.uint8).reshape(K, lam)
        y = d.eval_multikey_device(bool(b), torch.frombuffer(bytearray(cwb), dtype=torch.uint8).cuda(),
                                   torch.from_numpy(s0s.copy()).cuda(), torch.from_numpy(xs).cuda(), Pk)
        torch.cuda.synchronize()
        got = y.cpu().numpy()
        for k in range(K):
            want = O.eval_(P, b, oks[k], S[k].tobytes(), xs[k * Pk:(k + 1) * Pk])
            assert np.array_equal(got[k * Pk:(k + 1) * Pk], want), (b, k)
