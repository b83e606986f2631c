"""Latency kernels (kernels_lat.h: one AES column per lane) and concurrent use of one
dcf_prg (include/dcf_hip.h "Threading"), on the GPU, byte-identical to the oracle.

* k_eval16_row (32 lanes per point, one lookup per lane and round) serves auto-mode
  single-key eval up to kEvalRowMax points and k_eval16_oct (8 lanes per point) up to
  kEvalOctMax points, through the device entry point and through the host entry
  point's tiny path (the kernel reads the key and points from, and writes the outputs
  to, mapped pinned memory); k_gen16_col (16 lanes per key) serves gen up to
  kGenColMax keys (dcf_gen and dcf_gen_batch_device).
* One prg shared by 8 host threads (the reference's `&self` + `Prg: Sync`, lib.rs:34,52),
  each thread with its own key and points, host and device entry points mixed; and a host
  call queued right after a device call on the same prg with no synchronize in between
  (the host call must be ordered after the device call's kernels).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
CPU_THREADS = 16


@pytest.fixture(scope="module")
def dcf(hip_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import dcf_amd
    return dcf_amd


def _T(b):
    import torch
    return torch.from_numpy(np.frombuffer(bytes(b), np.uint8).copy()).cuda()


@pytest.mark.parametrize("nb", [1, 3, 4, 16, 32])
@pytest.mark.parametrize("m", [1, 2, 31, 33, 127, 128, 129, 2048, 8192, 8193, 12000])
def test_oct_eval_vs_oracle(dcf, nb, m):
    import torch
    rng = np.random.default_rng(nb * 1000 + m)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    bound = m % 2
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(bound))
    ok = O.gen(P, alpha, beta, s0, s1, bound)
    assert [cw.s for cw in k.cws] == [bytes(r) for r in ok.cw_s] and k.cw_np1 == bytes(ok.cw_np1)
    xs = rng.integers(0, 256, (m, nb), dtype=np.uint8)
    xs[0] = np.frombuffer(alpha, np.uint8)  # the boundary point itself
    # bit patterns that drive each slot case of k_eval16_oct's schedule: runs of right steps
    # (0xff), left steps (0x00), (R, L) pairs back to back (0xaa: the deferred-B queue full at
    # every other pair), (L, R) (0x55), long runs ending at a word edge (0x0f / 0xf0), x ending
    # in a right step (last level paired with a deferred B or alone)
    pats = [b"\xff", b"\x00", b"\xaa", b"\x55", b"\x0f", b"\xf0", b"\x33", b"\xcc", b"\x01", b"\x80"]
    for i, pt in enumerate(pats[:max(0, m - 1)]):
        xs[1 + i] = np.frombuffer(pt * nb, np.uint8)
    cwb = dcf.share_to_cwb(k, nb, 16)
    for b, sb in ((0, s0), (1, s1)):
        want = O.eval_(P, b, ok, sb, xs, nthreads=CPU_THREADS)
        got_h = d.eval(bool(b), dcf.Share([sb], k.cws, k.cw_np1), xs)           # host tiny path
        got_d = d.eval_device(bool(b), _T(cwb), _T(sb), torch.from_numpy(xs).cuda())  # device path
        torch.cuda.synchronize()
        assert np.array_equal(got_h, want), (nb, m, b)
        assert np.array_equal(got_d.cpu().numpy(), want), (nb, m, b)


@pytest.mark.parametrize("nb", [1, 2, 16, 32])
@pytest.mark.parametrize("K", [1, 5, 64, 65, 1024, 2048, 2049, 5000])
def test_col_gen_vs_oracle(dcf, nb, K):
    import torch
    rng = np.random.default_rng(nb * 7919 + K)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    d = dcf.DcfImpl(nb, 16, prg)
    A = rng.integers(0, 256, (K, nb), dtype=np.uint8)
    B, S0, S1 = (rng.integers(0, 256, (K, 16), dtype=np.uint8) for _ in range(3))
    bound = K % 2
    cwb = d.gen_batch_device(*(torch.from_numpy(a).cuda() for a in (A, B, S0, S1)), dcf.BoundState(bound))
    torch.cuda.synchronize()
    c = cwb.cpu().numpy()
    n = 8 * nb
    for key in sorted({0, K // 2, K - 1}):
        ok = O.gen(P, A[key].tobytes(), B[key].tobytes(), S0[key].tobytes(), S1[key].tobytes(), bound)
        assert np.array_equal(c[:n * K * 16].reshape(n, K, 16)[:, key], ok.cw_s)
        assert np.array_equal(c[n * K * 16:2 * n * K * 16].reshape(n, K, 16)[:, key], ok.cw_v)
        assert np.array_equal(c[2 * n * K * 16:2 * n * K * 16 + n * K].reshape(n, K)[:, key], ok.cw_t)
        off = dcf.cwb_np1_offset(nb, 16, K)
        assert np.array_equal(c[off:off + K * 16].reshape(K, 16)[key], ok.cw_np1)
    # one key through the host entry point (tiny path: mapped pinned buffer)
    k = d.gen(dcf.CmpFn(A[0].tobytes(), B[0].tobytes()), [S0[0].tobytes(), S1[0].tobytes()], dcf.BoundState(bound))
    ok = O.gen(P, A[0].tobytes(), B[0].tobytes(), S0[0].tobytes(), S1[0].tobytes(), bound)
    assert [cw.s for cw in k.cws] == [bytes(r) for r in ok.cw_s]
    assert [cw.v for cw in k.cws] == [bytes(r) for r in ok.cw_v]
    assert k.cw_np1 == bytes(ok.cw_np1)
    blob = dcf.share_to_cwb(k, nb, 16)
    pad = blob[2 * n * 16 + n:dcf.cwb_np1_offset(nb, 16, 1)]
    assert pad == bytes(len(pad))


def _job(dcf, prg, i, device_stream):
    """Thread i's own key and points on the shared prg: gen, three host evals and (every other
    thread) a device eval on a stream of its own; returns the inputs and outputs."""
    import torch
    rng = np.random.default_rng(500 + i)
    nb = (16, 4, 16, 2, 16, 8, 16, 1)[i % 8]
    m = (1, 1000, 70_000, 3, 300_000, 129, 5, 2048)[i % 8]
    d = dcf.DcfImpl(nb, 16, prg)
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState(i % 2))
    xs = rng.integers(0, 256, (m, nb), dtype=np.uint8)
    outs = []
    for rep in range(3):
        outs.append(d.eval(bool(i % 2), dcf.Share([s1 if i % 2 else s0], k.cws, k.cw_np1), xs))
    dev = None
    if device_stream:
        with torch.cuda.stream(torch.cuda.Stream()):
            yd = d.eval_device(bool(i % 2), _T(dcf.share_to_cwb(k, nb, 16)), _T(s1 if i % 2 else s0),
                               torch.from_numpy(xs).cuda())
            torch.cuda.current_stream().synchronize()
            dev = yd.cpu().numpy()
    return nb, alpha, beta, s0, s1, xs, outs, dev


def test_one_prg_many_threads(dcf):
    rng = np.random.default_rng(9)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(lambda i: _job(dcf, prg, i, i % 2 == 0), range(16)))
    assert prg.workspaces() >= 2  # calls really overlapped
    for i, (nb, alpha, beta, s0, s1, xs, outs, dev) in enumerate(res):
        ok = O.gen(P, alpha, beta, s0, s1, i % 2)
        idx = np.unique(np.concatenate([np.arange(min(len(xs), 400)), np.arange(max(0, len(xs) - 400), len(xs))]))
        want = O.eval_(P, i % 2, ok, s1 if i % 2 else s0, xs[idx], nthreads=CPU_THREADS)
        for o in outs:
            assert np.array_equal(o[idx], want), i
            assert np.array_equal(o, outs[0]), i
        if dev is not None:
            assert np.array_equal(dev, outs[0]), i
    # every workspace is idle now: trim frees them all, and the prg keeps working
    n = prg.workspaces()
    pinned = prg.host_pinned_bytes()
    assert pinned > 0 and prg.trim() == n and prg.workspaces() == 0 and prg.host_pinned_bytes() == 0
    nb, alpha, beta, s0, s1, xs, outs, dev = _job(dcf, prg, 3, False)
    ok = O.gen(P, alpha, beta, s0, s1, 1)
    assert np.array_equal(outs[0][:64], O.eval_(P, 1, ok, s1, xs[:64], nthreads=CPU_THREADS))
    assert prg.workspaces() == 1


def test_host_call_after_device_call_without_sync(dcf):
    """eval_device (2^22 points, shared-prefix table on the workspace) immediately followed by
    host-pointer eval and gen on the same prg: the host calls reuse the device call's workspace
    (LIFO pool) and must wait for its kernels instead of rebuilding its table under them."""
    import torch
    rng = np.random.default_rng(21)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    d = dcf.DcfImpl(16, 16, prg)
    ka = d.gen(dcf.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf.BoundState.LtBeta)
    kb = d.gen(dcf.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf.BoundState.GtBeta)
    xs = torch.from_numpy(rng.integers(0, 256, (1 << 22, 16), dtype=np.uint8)).cuda()
    cwa, sa = _T(dcf.share_to_cwb(ka, 16, 16)), _T(ka.s0s[0])
    ref = d.eval_device(False, cwa, sa, xs)
    torch.cuda.synchronize()
    got = d.eval_device(False, cwa, sa, xs)  # queued; no synchronize before the host calls
    xh = rng.integers(0, 256, (1 << 20, 16), dtype=np.uint8)
    yb = d.eval(True, dcf.Share([kb.s0s[1]], kb.cws, kb.cw_np1), xh)  # a depth-20 table in the same buffer
    d.gen(dcf.CmpFn(bytes(16), bytes(16)), [bytes(16), bytes(16)], dcf.BoundState.LtBeta)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    yb2 = d.eval(True, dcf.Share([kb.s0s[1]], kb.cws, kb.cw_np1), xh)
    assert np.array_equal(yb, yb2)
    kbo = O.OracleKey(16, 16)
    kbo.cw_s[:] = [np.frombuffer(cw.s, np.uint8) for cw in kb.cws]
    kbo.cw_v[:] = [np.frombuffer(cw.v, np.uint8) for cw in kb.cws]
    kbo.cw_t[:] = [int(cw.tl) | (int(cw.tr) << 1) for cw in kb.cws]
    kbo.cw_np1[:] = np.frombuffer(kb.cw_np1, np.uint8)
    assert np.array_equal(yb[:500], O.eval_(P, 1, kbo, kb.s0s[1], xh[:500], nthreads=CPU_THREADS))


def test_multikey_back_to_back_streams(dcf):
    """Multi-key evals queued on two streams with no synchronization between them: the second call
    reuses the first's workspace (LIFO pool), whose per-key top trees it rebuilds on the workspace's
    second stream — that build must wait for the first call's walk (fork / join events)."""
    import torch
    rng = np.random.default_rng(41)
    keys = [rng.bytes(32) for _ in range(2)]
    prg, P = dcf.Aes256HirosePrg(keys, 16), O.OraclePrg(keys, 16)
    d = dcf.DcfImpl(16, 16, prg)
    K, Pp = 3000, 64
    sets = []
    for j in range(2):
        alpha, beta, s0, s1 = (rng.integers(0, 256, (K, w), dtype=np.uint8) for w in (16, 16, 16, 16))
        cwb = d.gen_batch_device(_T(alpha.tobytes()).view(K, 16), _T(beta.tobytes()).view(K, 16),
                                 _T(s0.tobytes()).view(K, 16), _T(s1.tobytes()).view(K, 16), dcf.BoundState(j))
        xs = torch.from_numpy(rng.integers(0, 256, (K * Pp, 16), dtype=np.uint8)).cuda()
        sets.append((alpha, beta, s0, s1, cwb, xs))
    refs = []
    for alpha, beta, s0, s1, cwb, xs in sets:
        refs.append(d.eval_multikey_device(False, cwb, _T(s0.tobytes()).view(K, 16), xs, Pp))
        torch.cuda.synchronize()
    got = []
    for (alpha, beta, s0, s1, cwb, xs), st in zip(sets, (torch.cuda.Stream(), torch.cuda.Stream())):
        with torch.cuda.stream(st):
            got.append(d.eval_multikey_device(False, cwb, _T(s0.tobytes()).view(K, 16), xs, Pp))
    torch.cuda.synchronize()
    for j, (alpha, beta, s0, s1, cwb, xs) in enumerate(sets):
        assert torch.equal(got[j], refs[j]), j
        for key in (0, K // 2, K - 1):
            ok = O.gen(P, alpha[key].tobytes(), beta[key].tobytes(), s0[key].tobytes(), s1[key].tobytes(), j)
            sl = slice(key * Pp, (key + 1) * Pp)
            want = O.eval_(P, 0, ok, s0[key].tobytes(), xs[sl].cpu().numpy())
            assert np.array_equal(refs[j][sl].cpu().numpy(), want), (j, key)


def test_phase_timing(dcf):
    import torch
    rng = np.random.default_rng(3)
    prg = dcf.Aes256HirosePrg([rng.bytes(32) for _ in range(2)], 16)
    d = dcf.DcfImpl(16, 16, prg)
    k = d.gen(dcf.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf.BoundState.LtBeta)
    xs = torch.from_numpy(rng.integers(0, 256, (1 << 21, 16), dtype=np.uint8)).cuda()
    with pytest.raises(dcf.DcfError):
        prg.last_eval_phases()
    prg.set_phase_timing(True)
    y = d.eval_device(False, _T(dcf.share_to_cwb(k, 16, 16)), _T(k.s0s[0]), xs)
    torch.cuda.synchronize()
    prep, walk, depth = prg.last_eval_phases()
    assert depth == prg.eval_prefix_levels(16, 1, 1 << 21) == 21
    assert 0 < prep < walk
    prg.set_phase_timing(False)
    y2 = d.eval_device(False, _T(dcf.share_to_cwb(k, 16, 16)), _T(k.s0s[0]), xs)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
