"""The multi-process path on the GPU box through the HIP library: two ranks (gloo, both on
cuda:0 — RCCL needs one GPU per rank), key broadcast from rank 0, an ODD number of points
split by point_slice (the slices differ by one point), each rank evaluating its slice with
dcf_eval_device, and gather_shares onto rank 0.  The gathered shares must be byte-identical
to one dcf_eval_device over every point (the reference writes all outputs into the
caller's ys, lib.rs:163,196-198)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, out_path, total, nb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    import dcf_amd
    from dcf_amd.dist import broadcast_key, gather_shares, point_slice
    lam = 16
    rng = np.random.default_rng(31)
    keys = [rng.bytes(32) for _ in range(2)]
    d = dcf_amd.DcfImpl(nb, lam, dcf_amd.Aes256HirosePrg(keys, lam))
    cwb = torch.zeros(dcf_amd.cwb_bytes(nb, lam, 1), dtype=torch.uint8, device="cuda")
    seeds = torch.zeros((2, lam), dtype=torch.uint8, device="cuda")
    if rank == 0:  # only rank 0 runs gen (on its GPU)
        s0, s1 = rng.bytes(lam), rng.bytes(lam)
        k = d.gen(dcf_amd.CmpFn(rng.bytes(nb), rng.bytes(lam)), [s0, s1], dcf_amd.BoundState.LtBeta)
        cwb.copy_(torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, nb, lam), np.uint8).copy()))
        seeds.copy_(torch.from_numpy(np.frombuffer(s0 + s1, np.uint8).reshape(2, lam).copy()))
    broadcast_key([cwb, seeds])
    g = torch.Generator(device="cuda")
    g.manual_seed(99)
    xs_all = torch.randint(0, 256, (total, nb), dtype=torch.uint8, device="cuda", generator=g)
    start, cnt = point_slice(total, ws, rank)
    ys = d.eval_device(True, cwb, seeds[1].contiguous(), xs_all[start:start + cnt].contiguous())
    torch.cuda.synchronize()
    full = gather_shares(ys)
    if rank == 0:
        ref = d.eval_device(True, cwb, seeds[1].contiguous(), xs_all)
        torch.cuda.synchronize()
        np.save(out_path, np.stack([full.cpu().numpy(), ref.cpu().numpy()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("total,nb", [(1_000_003, 16), (4097, 4)])
def test_two_rank_hip_eval_gather_odd_total(tmp_path, total, nb):
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(2, _free_port(), out, total, nb), nprocs=2, join=True)
    full, ref = np.load(out)
    assert full.shape == (total, 16)
    assert np.array_equal(full, ref)


def _rccl_worker(rank, port, out_path, total, nb):
    """World size 1 over RCCL (backend "nccl"): the same broadcast / gather / object
    all-gather calls an 8-GPU run makes, on GPU tensors, so RCCL itself executes here."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    import dcf_amd
    from dcf_amd.dist import broadcast_key, gather_shares, point_slice
    lam = 16
    rng = np.random.default_rng(47)
    keys = [rng.bytes(32) for _ in range(2)]
    d = dcf_amd.DcfImpl(nb, lam, dcf_amd.Aes256HirosePrg(keys, lam))
    s0, s1 = rng.bytes(lam), rng.bytes(lam)
    k = d.gen(dcf_amd.CmpFn(rng.bytes(nb), rng.bytes(lam)), [s0, s1], dcf_amd.BoundState.LtBeta)
    cwb_src = torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, nb, lam), np.uint8).copy()).cuda()
    seeds_src = torch.from_numpy(np.frombuffer(s0 + s1, np.uint8).reshape(2, lam).copy()).cuda()
    cwb, seeds = cwb_src.clone(), seeds_src.clone()
    broadcast_key([cwb, seeds])                       # ncclBroadcast (root 0)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    xs = torch.randint(0, 256, (total, nb), dtype=torch.uint8, device="cuda", generator=g)
    start, cnt = point_slice(total, 1, 0)
    ys = d.eval_device(False, cwb, seeds[0].contiguous(), xs[start:start + cnt].contiguous())
    full = gather_shares(ys)                          # row-count all_gather + ncclGather on GPU tensors
    objs = [None]
    dist.all_gather_object(objs, {"rank": 0, "rows": int(ys.shape[0])})
    ref = d.eval_device(False, cwb_src, seeds_src[0].contiguous(), xs)
    torch.cuda.synchronize()
    np.save(out_path, np.stack([full.cpu().numpy(), ref.cpu().numpy()]))
    assert torch.equal(cwb, cwb_src) and torch.equal(seeds, seeds_src)
    assert full.is_cuda and objs == [{"rank": 0, "rows": total}]
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_world1_broadcast_gather_identical():
    """RCCL executes (nccl backend, world 1): broadcast_key, gather_shares on GPU tensors and
    all_gather_object; the gathered shares equal one dcf_eval_device byte for byte."""
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "res.npy")
        mp.spawn(_rccl_worker, args=(_free_port(), out, 300_007, 16), nprocs=1, join=True)
        full, ref = np.load(out)
    assert full.shape == (300_007, 16)
    assert np.array_equal(full, ref)
