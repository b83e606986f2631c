"""Host-pointer pipeline and the multi-GPU C ABI (dcf_eval_multi_gpu[_device]).

On the 1-GPU box, G "devices" are G distinct dcf_prg objects on device 0 (each with
its own workspaces: streams, staging and work counter): slice placement, per-slice key
copies, the threads of the host variant and the gather are exercised exactly as on 8
GPUs; only the peer copy degenerates to a device-local one — the cross-device branch of
dcf_eval_multi_gpu_device (hipDeviceEnablePeerAccess + hipMemcpyPeerAsync over xGMI) is
NOT executed on this box and is untested here.  Every result must be
byte-identical to dcf_eval_device over the whole batch (the reference
splits Dcf::eval over host cores inside one call, lib.rs:194-199).
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

CPU_THREADS = 16


def test_point_slice_matches_dist_helper(hip_lib):
    from dcf_amd import point_slice
    from dcf_amd.dist import point_slice as py_slice
    for total in (0, 1, 7, 64, 1001, 1 << 28):
        for G in (1, 2, 3, 8):
            got = [point_slice(total, G, g) for g in range(G)]
            assert got == [py_slice(total, G, g) for g in range(G)]
            assert sum(c for _, c in got) == total
    assert point_slice(10, 2, 5) == (10, 0)


def test_multi_gpu_argument_validation_without_gpu(hip_lib):
    L = hip_lib
    arr = (ctypes.c_void_p * 2)(None, None)
    assert L.dcf_eval_multi_gpu(None, 0, 16, 0, None, 0, None, None, 0, None, 0) == -1
    assert L.dcf_eval_multi_gpu(arr, 2, 16, 0, None, 0, None, None, 0, None, 0) == -1
    assert L.dcf_eval_multi_gpu_device(arr, 2, 16, 0, None, 0, None, None, None, None, None, None) == -1


class _StubPrg:
    """Stands in for a prg so the Python-side checks run without a GPU: they must reject
    bad buffers before any pointer reaches the C ABI."""
    lam, device = 16, 0
    handle = ctypes.c_void_p(0)


def test_device_entry_points_reject_bad_tensors_without_gpu(hip_lib):
    import torch
    import dcf_amd
    d = dcf_amd.DcfImpl.__new__(dcf_amd.DcfImpl)
    d.n_bytes, d.lam, d.prg = 16, 16, _StubPrg()
    cwb = torch.zeros(dcf_amd.cwb_bytes(16, 16, 1), dtype=torch.uint8)
    s0 = torch.zeros(16, dtype=torch.uint8)
    xs = torch.zeros((8, 16), dtype=torch.uint8)
    for bad_xs in (xs.to(torch.int64), xs, xs.t()):  # wrong dtype / host tensor / non-contiguous
        with pytest.raises(dcf_amd.DcfError) as e:
            d.eval_device(False, cwb, s0, bad_xs)
        assert e.value.code == -1
    with pytest.raises(dcf_amd.DcfError):
        d.eval_multikey_device(False, cwb, s0.view(1, 16), xs, 8)
    with pytest.raises(dcf_amd.DcfError):
        d.gen_batch_device(xs, xs, xs, xs, dcf_amd.BoundState.LtBeta)
    with pytest.raises(dcf_amd.DcfError):
        d.eval_full_domain_device(False, cwb, s0)
    with pytest.raises(dcf_amd.DcfError):
        d.eval_device(False, np.zeros(4240, np.uint8), s0, xs)


@pytest.fixture(scope="module")
def dcf(hip_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import dcf_amd
    return dcf_amd


def _key(dcf, nb, lam, cipher_n, seed):
    rng = np.random.default_rng(seed)
    keys = [rng.bytes(32) for _ in range(cipher_n)]
    alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    return rng, keys, alpha, beta, s0, s1


@pytest.mark.gpu
@pytest.mark.parametrize("nb,lam,m", [(16, 16, 9_000_001), (4, 16, (1 << 22) + 3), (16, 16384, 20_000),
                                      (3, 16, 1), (16, 16, 257)])
def test_host_path_chunked_pipeline(dcf, nb, lam, m):
    """dcf_eval (host buffers) through the 3-stream chunked pipeline: 128 MiB chunks, so
    9M points at N = LAMBDA = 16 run 3 chunks (ragged last), 20k points at LAMBDA = 16384
    run 3 chunks of 8184; must equal the device path over the whole batch."""
    import torch
    rng, keys, alpha, beta, s0, s1 = _key(dcf, nb, lam, 2 if lam == 16 else 18, nb * 7 + m)
    prg = dcf.Aes256HirosePrg(keys, lam)
    d = dcf.DcfImpl(nb, lam, prg)
    k = d.gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.GtBeta)
    xs = rng.integers(0, 256, (m, nb), dtype=np.uint8)
    y = d.eval(True, dcf.Share([s1], k.cws, k.cw_np1), xs)
    T = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()  # noqa: E731
    yd = d.eval_device(True, T(dcf.share_to_cwb(k, nb, lam)), T(s1), torch.from_numpy(xs).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(y, yd.cpu().numpy())
    P = O.OraclePrg(keys, lam)
    ok = O.gen(P, alpha, beta, s0, s1, 1)
    idx = np.unique(np.concatenate([np.arange(min(m, 300)), np.arange(max(0, m - 300), m)]))
    assert np.array_equal(y[idx], O.eval_(P, 1, ok, s1, xs[idx], nthreads=CPU_THREADS))


@pytest.mark.gpu
@pytest.mark.parametrize("G,nb,lam,m", [(2, 16, 16, 1_000_003), (3, 4, 16, 5_000_000), (8, 16, 16, 100_000),
                                        (2, 16, 1024, 3001), (4, 2, 16, 3)])
def test_eval_multi_gpu_host_and_device(dcf, G, nb, lam, m):
    """G dcf_prg (same keys) on device 0: the host variant (one thread per prg) and the
    device variant (per-slice buffers, key copied per device, gather into one buffer)
    both equal dcf_eval_device over the whole batch.  G = 4 with 3 points leaves a
    slice empty."""
    import torch
    rng, keys, alpha, beta, s0, s1 = _key(dcf, nb, lam, 2 if lam == 16 else 18, G * 100 + nb)
    impls = [dcf.DcfImpl(nb, lam, dcf.Aes256HirosePrg(keys, lam)) for _ in range(G)]
    k = impls[0].gen(dcf.CmpFn(alpha, beta), [s0, s1], dcf.BoundState.LtBeta)
    cwb = dcf.share_to_cwb(k, nb, lam)
    xs = rng.integers(0, 256, (m, nb), dtype=np.uint8)
    T = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()  # noqa: E731
    xs_d = torch.from_numpy(xs).cuda()
    want = impls[0].eval_device(False, T(cwb), T(s0), xs_d)
    torch.cuda.synchronize()
    want_h = want.cpu().numpy()
    md = dcf.MultiGpuDcf(impls)
    got = md.eval(False, dcf.Share([s0], k.cws, k.cw_np1), xs)
    assert np.array_equal(got, want_h)
    slices = [dcf.point_slice(m, G, g) for g in range(G)]
    xsl = [xs_d[st:st + c] for st, c in slices]
    gather = torch.empty((m, lam), dtype=torch.uint8, device="cuda")
    ysl = md.eval_device(False, cwb, s0, xsl, gather=gather)
    for (st, c), y in zip(slices, ysl):
        assert torch.equal(y, want[st:st + c])
    assert torch.equal(gather, want)


@pytest.mark.gpu
def test_eval_multi_gpu_rejects_mismatched_prgs(dcf):
    keys = [bytes([1]) * 32, bytes([2]) * 32]
    a = dcf.DcfImpl(16, 16, dcf.Aes256HirosePrg(keys, 16))
    b = dcf.DcfImpl(16, 16, dcf.Aes256HirosePrg([bytes([3]) * 32, bytes([2]) * 32], 16))
    k = a.gen(dcf.CmpFn(bytes(16), bytes(16)), [bytes(16), bytes(16)], dcf.BoundState.LtBeta)
    xs = np.zeros((10, 16), np.uint8)
    with pytest.raises(dcf.DcfError) as e:
        dcf.MultiGpuDcf([a, b]).eval(False, k, xs)  # different PRG keys
    assert e.value.code == -1
    with pytest.raises(dcf.DcfError):
        dcf.MultiGpuDcf([a, a]).eval(False, k, xs)  # one prg twice
    with pytest.raises(dcf.DcfError) as e:
        dcf.MultiGpuDcf([a]).eval(False, k, xs, np.zeros((9, 16), np.uint8))
    assert e.value.code == -5


@pytest.mark.gpu
def test_device_entry_points_reject_bad_shapes(dcf):
    """row widths and buffer sizes are checked before the C ABI (which takes
    no lengths for device buffers)."""
    import torch
    prg = dcf.Aes256HirosePrg([bytes(32)] * 2, 16)
    d = dcf.DcfImpl(16, 16, prg)
    cwb = torch.zeros(dcf.cwb_bytes(16, 16, 1), dtype=torch.uint8, device="cuda")
    s0 = torch.zeros(16, dtype=torch.uint8, device="cuda")
    xs = torch.zeros((64, 16), dtype=torch.uint8, device="cuda")
    cases = [
        lambda: d.eval_device(False, cwb, s0, xs[:, :15].contiguous()),   # N - 1 columns
        lambda: d.eval_device(False, cwb[:-1], s0, xs),                     # short key
        lambda: d.eval_device(False, cwb, s0[:8], xs),                      # short seed
        lambda: d.eval_device(False, cwb, s0, xs, torch.empty((63, 16), dtype=torch.uint8, device="cuda")),
        lambda: d.eval_multikey_device(False, cwb, s0.view(1, 16), xs, 32),  # rows != K * P
        lambda: d.gen_batch_device(xs, xs, xs, xs[:63].contiguous(), dcf.BoundState.LtBeta),
        lambda: d.eval_device(False, cwb, s0, xs.to(torch.int32)),
    ]
    for f in cases:
        with pytest.raises(dcf.DcfError):
            f()


@pytest.mark.gpu
def test_prefix_memory_cap_and_device_bytes(dcf):
    """dcf_prg_set_prefix_max_bytes lowers the AUTO shared-prefix depth until its buffers fit
    (none below depth 8), forced depths ignore it, output bytes never change;
    dcf_prg_device_bytes reports the resident table."""
    import torch
    rng = np.random.default_rng(77)
    keys = [rng.bytes(32) for _ in range(2)]
    prg = dcf.Aes256HirosePrg(keys, 16)
    d = dcf.DcfImpl(16, 16, prg)
    assert prg.eval_prefix_levels(16, 1, 1 << 28) == 27
    prg.set_prefix_max_bytes(1 << 30)
    # depth 24: 0.61e9 B fits 1 GiB, depth 25 (1.21e9 B) does not (include/dcf_hip.h sizes)
    assert prg.eval_prefix_levels(16, 1, 1 << 28) == 24
    prg.set_prefix_max_bytes(1000)
    assert prg.eval_prefix_levels(16, 1, 1 << 28) == 0
    prg.set_prefix_levels(12)
    assert prg.eval_prefix_levels(16, 1, 1 << 28) == 12   # forced: not capped
    prg.set_prefix_levels(-1)
    k = d.gen(dcf.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf.BoundState.LtBeta)
    T = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()  # noqa: E731
    xs = torch.from_numpy(rng.integers(0, 256, (1 << 20, 16), dtype=np.uint8)).cuda()
    cwb, s0 = T(dcf.share_to_cwb(k, 16, 16)), T(k.s0s[0])
    capped = d.eval_device(False, cwb, s0, xs)            # cap 1000 B: no table
    torch.cuda.synchronize()
    small = prg.device_bytes()
    prg.set_prefix_max_bytes(0)
    free = d.eval_device(False, cwb, s0, xs)              # auto depth 20
    torch.cuda.synchronize()
    assert torch.equal(capped, free)
    assert prg.device_bytes() >= small + (1 << 20) * 32   # the 2^20-row table is resident


def prefix_bytes_header(D: int) -> int:
    """Resident bytes of a Hirose LAMBDA = 16 shared-prefix table of depth D as include/dcf_hip.h
    states them: 32 * 2^D rows + the build's two node buffers 2 * 33 * 2^(D - H), H = min(4, D - 18)."""
    H = min(4, D - 18) if D > 18 else 0
    return 32 * 2 ** D + (2 * 33 * 2 ** (D - H) if H else 33 * 2 ** D)


@pytest.mark.gpu
def test_prefix_table_resident_bytes_c3(dcf):
    """After one auto-depth eval of 2^28 points (C3, D = 27) the prg holds the table and its
    build buffers (4.85e9 B, include/dcf_hip.h) plus small per-workspace scratch — no more —
    and dcf_prg_trim releases them."""
    import torch
    rng = np.random.default_rng(78)
    keys = [rng.bytes(32) for _ in range(2)]
    prg = dcf.Aes256HirosePrg(keys, 16)
    d = dcf.DcfImpl(16, 16, prg)
    k = d.gen(dcf.CmpFn(rng.bytes(16), rng.bytes(16)), [rng.bytes(16), rng.bytes(16)], dcf.BoundState.LtBeta)
    T = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()  # noqa: E731
    cwb, s0 = T(dcf.share_to_cwb(k, 16, 16)), T(k.s0s[0])
    base = prg.device_bytes()
    m = 1 << 28
    assert prg.eval_prefix_levels(16, 1, m) == 27
    xs = torch.zeros((m, 16), dtype=torch.uint8, device="cuda")
    ys = d.eval_device(False, cwb, s0, xs)
    torch.cuda.synchronize()
    held = prg.device_bytes() - base
    want = prefix_bytes_header(27)
    assert want == 4_848_615_424
    assert want <= held <= want + (64 << 20), (held, want)
    del xs, ys
    assert prg.trim() >= 1
    assert prg.device_bytes() <= base + (1 << 20)

