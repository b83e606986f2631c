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


def _no_launcher_env():
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _one_line(out):
    lines = out.stdout.strip().splitlines()
    assert len(lines) == 1, out.stdout[:2000]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_no_launcher_two_ranks_and_multi_gpu_abi():
    """`python bench.py --gpus 2` with no launcher (the driver's BENCH command form): bench.py
    starts the two ranks itself, stdout is exactly the one JSON line, the slices match, and
    rank 0's one-process multi-GPU ABI check (dcf_eval_multi_gpu_device + gather) matches its
    own dcf_eval_device."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--points", str((1 << 22) + 3), "--no-cpu", "--no-compare", "--dist-backend", "gloo", "--check"]
    out = subprocess.run(cmd, cwd=ROOT, env=_no_launcher_env(), capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _one_line(out)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["slice_check"]["slices_match"], d["slice_check"]
    assert [r["rank"] for r in d["per_rank"]["ranks"]] == [0, 1]
    abi = d["multi_gpu_abi_check"]
    assert abi["ok"], abi
    assert len(abi["devices"]) >= 2 and abi["slices_match"] and abi["gather_matches"]


@pytest.mark.gpu
def test_bench_c5_two_ranks_check():
    """C5's N > 1 path: 2 ranks (no launcher), keys split over the ranks (odd total), rank 0
    regenerates every rank's keys and points, re-runs gen + both parties' eval and compares
    digests; the per-rank block covers both ranks' keys."""
    keys = 4099
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c5", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--keys", str(keys), "--no-cpu", "--dist-backend", "gloo", "--check"]
    out = subprocess.run(cmd, cwd=ROOT, env=_no_launcher_env(), capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _one_line(out)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "strong"
    assert d["slice_check"]["slices_match"], d["slice_check"]
    pr = d["per_rank"]["ranks"]
    assert [r["rank"] for r in pr] == [0, 1]
    assert sum(r["keys"] for r in pr) == keys and [r["key_start"] for r in pr] == [0, 2050]
    for r in pr:
        assert r["gen_ms"] > 0 and r["eval_ms"] > 0


def test_spawn_ranks_env_and_exit_status(capfd):
    """bench.spawn_ranks (no launcher): every rank gets the launcher's environment, and a failing
    rank ends the others and sets the exit status (CPU only: the ranks here run a stub)."""
    import bench
    env = _no_launcher_env()
    code = ("import os; print('R', os.environ['RANK'], os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], "
            "os.environ['MASTER_ADDR'], os.environ['MASTER_PORT'], flush=True)")
    assert bench.spawn_ranks(3, [sys.executable, "-c", code], env=env) == 0
    got = sorted(ln.split() for ln in capfd.readouterr().out.splitlines() if ln.startswith("R "))
    assert [g[1:5] for g in got] == [[str(r), str(r), "3", "127.0.0.1"] for r in range(3)]
    assert len({g[5] for g in got}) == 1
    # rank 1 fails at once; rank 0 would sleep for a minute but is ended
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(60) if r == 0 else sys.exit(3)"
    import time
    t0 = time.perf_counter()
    assert bench.spawn_ranks(2, [sys.executable, "-c", code], env=env) == 3
    assert time.perf_counter() - t0 < 30


@pytest.mark.gpu
def test_bench_c4_two_ranks_check():
    """C4's N > 1 path (north_star: 2^22 points PER GPU, weak scaling, LAMBDA = 16384): 2 ranks
    (no launcher), each rank its own point range, rank 0 regenerates both ranks' points and
    compares output digests, and the one-process multi-GPU ABI check runs at LAMBDA = 16384."""
    pts = 4099
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c4", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--points", str(pts), "--no-cpu", "--no-compare", "--dist-backend", "gloo", "--check"]
    out = subprocess.run(cmd, cwd=ROOT, env=_no_launcher_env(), capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _one_line(out)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["lambda"] == 16384 and d["config"]["points_per_gpu"] == pts
    assert d["config"]["global_points"] == 2 * pts
    assert d["slice_check"]["slices_match"], d["slice_check"]
    pr = d["per_rank"]["ranks"]
    assert [r["rank"] for r in pr] == [0, 1]
    assert [r["start"] for r in pr] == [0, pts] and all(r["points"] == pts for r in pr)
    for r in pr:
        assert r["kernel_ms"] > 0 and r["walk_ms"] > 0
    abi = d["multi_gpu_abi_check"]
    assert abi["ok"], abi
    assert len(abi["devices"]) >= 2 and abi["slices_match"] and abi["gather_matches"]
