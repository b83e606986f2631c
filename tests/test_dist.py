"""Multi-process path on CPU (gloo, world_size 2): key broadcast, point
sharding and share gathering reproduce the single-process evaluation exactly.
The per-rank compute here is the oracle (no GPU in this container); on MI355X
the same plumbing drives libdcf_hip.so (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dcf_amd.dist import broadcast_key, gather_shares, point_slice, weak_slice


def test_point_slice_covers_exactly():
    for total in (0, 1, 7, 64, 1001):
        for ws in (1, 2, 3, 8):
            got = [point_slice(total, ws, r) for r in range(ws)]
            assert sum(c for _, c in got) == total
            assert all(got[r][0] + got[r][1] == got[r + 1][0] for r in range(ws - 1))
    assert weak_slice(100, 3) == (300, 100)
    with pytest.raises(ValueError):
        point_slice(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, out_path, total, pass_counts):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from oracle import oracle as O
    keys = [bytes([7]) * 32, bytes([9]) * 32]
    P = O.OraclePrg(keys, 16)
    nb, lam = 4, 16
    n = 8 * nb
    cwb = torch.zeros(2 * n * lam + n + lam, dtype=torch.uint8)
    seeds = torch.zeros((2, lam), dtype=torch.uint8)
    if rank == 0:  # only rank 0 runs gen
        rng = np.random.default_rng(5)
        s0, s1 = rng.bytes(lam), rng.bytes(lam)
        k = O.gen(P, b"\x12\x34\x56\x78", rng.bytes(lam), s0, s1, 0)
        blob = k.cw_s.tobytes() + k.cw_v.tobytes() + k.cw_t.tobytes() + k.cw_np1.tobytes()
        cwb.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
        seeds.copy_(torch.frombuffer(bytearray(s0 + s1), dtype=torch.uint8).view(2, lam))
    broadcast_key([cwb, seeds])
    k = O.OracleKey(nb, lam)
    c = cwb.numpy()
    k.cw_s[:] = c[:n * lam].reshape(n, lam)
    k.cw_v[:] = c[n * lam:2 * n * lam].reshape(n, lam)
    k.cw_t[:] = c[2 * n * lam:2 * n * lam + n]
    k.cw_np1[:] = c[2 * n * lam + n:]
    xs_all = np.random.default_rng(11).integers(0, 256, (total, nb), dtype=np.uint8)
    start, cnt = point_slice(total, ws, rank)  # uneven when total % ws != 0
    ys = O.eval_(P, 0, k, seeds[0].numpy().tobytes(), xs_all[start:start + cnt]).reshape(cnt, lam)
    counts = [point_slice(total, ws, r)[1] for r in range(ws)] if pass_counts else None
    full = gather_shares(torch.from_numpy(ys), counts=counts)
    if rank == 0:
        ref = O.eval_(P, 0, k, seeds[0].numpy().tobytes(), xs_all)
        np.save(out_path, np.stack([full.numpy(), ref]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,total,pass_counts", [(2, 203, False), (2, 1, False), (3, 101, True)])
def test_bcast_shard_gather_uneven(tmp_path, ws, total, pass_counts):
    """Odd totals: the slices differ in length (and one is empty at total = 1); the gather
    pads and trims, so the concatenation equals one process's eval of every point."""
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(ws, _free_port(), out, total, pass_counts), nprocs=ws, join=True)
    full, ref = np.load(out)
    assert np.array_equal(full, ref)
