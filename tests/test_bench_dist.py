"""bench.py's multi-rank path on the GPU box: two ranks launched exactly as the driver
launches N > 1 (torch.distributed.run, 127.0.0.1), here on one device with the gloo
backend (RCCL needs one GPU per rank).  Key broadcast from rank 0, strong-scaled point
slices (dcf_point_slice), max-over-ranks timing, and --check: rank 0 re-evaluates both
slices and compares output digests."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_two_ranks_strong_scaling_check():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--points", str((1 << 22) + 3), "--no-cpu",
           "--no-compare", "--dist-backend", "gloo", "--check"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_points"] == (1 << 22) + 3
    assert d["config"]["points_per_gpu"] in ((1 << 21) + 1, (1 << 21) + 2)
    assert d["value"] > 0
    assert d["slice_check"]["slices_match"], d["slice_check"]
    # the N > 1 line explains a scaling curve: per-rank kernel / wall / table-build times
    pr = d["per_rank"]
    assert [r["rank"] for r in pr["ranks"]] == [0, 1]
    assert sum(r["points"] for r in pr["ranks"]) == (1 << 22) + 3
    for r in pr["ranks"]:
        assert r["kernel_ms"] > 0 and r["walk_ms"] > 0 and r["table_ms"] >= 0 and r["prefix_levels"] == 21
    assert pr["imbalance"] >= 1.0
    assert d["key_broadcast"]["ms"] is not None and d["key_broadcast"]["bytes"] > 0


@pytest.mark.gpu
def test_bench_rccl_world1_line():
    """bench.py at N = 1 with --force-dist over RCCL: the key broadcast, the timing all-reduce,
    the per-rank all_gather_object and --check's digest gather all go through RCCL, and the
    line says so (key_broadcast.backend == "nccl")."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--points", str((1 << 22) + 3), "--no-cpu",
           "--no-compare", "--dist-backend", "nccl", "--force-dist", "--check"]
    out = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ), capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    # stdout is the one JSON line (RCCL's banner at communicator init goes to stderr)
    assert len(out.stdout.strip().splitlines()) == 1, out.stdout[:2000]
    d = json.loads(out.stdout)
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["key_broadcast"]["backend"] == "nccl" and d["key_broadcast"]["bytes"] > 0
    assert d["slice_check"]["slices_match"]
    assert [r["rank"] for r in d["per_rank"]["ranks"]] == [0]
