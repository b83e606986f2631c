"""Benchmark: DCF batch eval on MI355X (BASELINE.json metric).

Workload (default, BASELINE.json configs[2] = SURVEY.md §8 C3): N = 16 (128-bit
x), LAMBDA = 16, Aes256HirosePrg, one key, 2^28 uniformly random points resident
in HBM, party 0 (the reference bench's shape, benches/dcf_batch_eval.rs:25-30,
scaled up).  A step = one `Dcf::eval` pass over the rank's points.  C3 is "a
single key at 2^28 points sharded across 1/2/4/8 MI355X": by default the 2^28
points are split into contiguous per-rank slices (strong scaling, dcf_point_slice);
`--scaling weak` gives every rank its own 2^28 points instead.  The key is
generated once on rank 0 and broadcast over RCCL before timing; there is no
collective inside the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c2|c3|c4|c5|fd|lat]
                  [--scaling strong|weak] [--host-path]
  torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement" for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import dcf_amd  # noqa: E402
from dcf_amd.dist import broadcast_key, point_slice, weak_slice  # noqa: E402

METRIC = "DCF evals/sec (node) at 128-bit input, λ=16B; AES blocks/s vs INT roofline"

# ---- roofline constants (MI355X_MICROARCH.md; op counts from the gfx950 disassembly) ----
CUS, CLK_HZ = 256, 2.4e9
LDS_LOOKUPS = CUS * 32 * CLK_HZ      # ds_read_b32: 64 lanes per 2 LDS cycles per CU (§LDS table)
VALU_OPS = CUS * 128 * CLK_HZ        # 4 SIMD-32 per CU, wave64 op every 2 cycles per SIMD
TT_LDS_PER_BLOCK = 14 * 16           # T-table AES-256: 16 lookups per round
TT_VALU_PER_BLOCK = 370              # 1 v_perm per lookup + 2 v_bitop3 per column + DCF share
PEAK_TT_BLOCKS = LDS_LOOKUPS / TT_LDS_PER_BLOCK  # ~87.8 G blocks/s: T-table alone is LDS-bound


ENGINE = {0: "stream", 1: "ttable", 4: "stream"}
KERNEL = {"ttable": "k_eval16", "ttable-small": "k_eval16_pair", "stream": "k_eval16_stream", "mmo": "k_eval16_mmo"}


# MMO (AES-128, kernels_mmo.h): 10 rounds x 16 lookups + 11 round-key ds_read_b128 (16 lanes/clk) per block
PEAK_MMO_BLOCKS = CUS * CLK_HZ / (160 / 32 + 11 / 16)
# Measured ceiling of the T-table AES-256 rounds alone on MI355X (scripts/micro/aes_rate.hip, r02):
# 74-75 G blocks/s for 1-4 blocks per lane, = 0.85 of PEAK_TT_BLOCKS (ds_read_b32 alone: 0.863).
MEASURED_TT_BLOCKS = 74.6e9
# ds_read_b32 issue alone (same micro-benchmark): 0.863 of the nominal rate — the LDS wall itself.
DS_READ_FRAC = 0.863


def measured_ceiling(achieved_blocks_per_s: float) -> dict:
    """The T-table AES rounds' practical ceiling beside the nominal LDS peak."""
    return {"value": MEASURED_TT_BLOCKS / 1e9, "unit": "G AES-256 blocks/s",
            "frac": achieved_blocks_per_s / MEASURED_TT_BLOCKS,
            "source": "scripts/micro/aes_rate.hip: T-table AES-256 rounds alone, 16 waves/CU (0.85 of peak)",
            "ds_read_ceiling": DS_READ_FRAC * PEAK_TT_BLOCKS / 1e9,
            "ds_read_frac": achieved_blocks_per_s / (DS_READ_FRAC * PEAK_TT_BLOCKS),
            "note": "the rounds-only micro-benchmark keeps every wave in the same phase; the engines "
                    "raise wave priority for their rounds (s_setprio, r05ae) and can exceed it — the "
                    "ds_read_b32 issue rate alone (ds_read_ceiling) is the wall"}


def engine_peak(engine: str) -> float:
    if engine in ("mmo", "mmo-wide"):
        return PEAK_MMO_BLOCKS
    return PEAK_TT_BLOCKS


def pmc_traffic(kernel: str, points: int, n_bytes: int, lam: int, prefix_levels: int = 0):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json: one entry per profiled launch shape, written by
    scripts/prof_summary.py from `scripts/gpu.sh TAG profile W`: 2 x FETCH_SIZE + WRITE_SIZE,
    MI355X_MICROARCH.md §HBM), only when a profile ran this exact launch shape; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    for e in (t if isinstance(t, list) else [t]):
        if (e.get("kernel"), e.get("points_per_launch"), e.get("n_bytes"), e.get("lambda"),
                e.get("prefix_levels", 0)) == (kernel, points, n_bytes, lam, prefix_levels):
            return e
    return None


def traffic_fields(kernel: str, points: int, n_bytes: int, lam: int, prefix_levels: int, alg_bytes: float):
    """(traffic, source): the PMC figure when profiles/ holds this launch shape, otherwise None
    (traffic is measured HBM bytes or nothing; the algorithmic bytes are in the line beside it)."""
    e = pmc_traffic(kernel, points, n_bytes, lam, prefix_levels)
    if e is not None and e.get("traffic_bytes") is not None:
        src = f"pmc: 2 x FETCH_SIZE + WRITE_SIZE per launch ({e.get('source', '?')}, via profiles/pmc_traffic.json)"
        if e.get("traffic_bytes_x1") is not None:
            src += (f"; 1 x FETCH_SIZE + WRITE_SIZE = {e['traffic_bytes_x1'] / 1e9:.2f} GB (the x2 correction is for "
                    f"wide streaming reads; 32-B row gathers are fetched as 64-B requests, so x1 may be the closer figure)")
        return e["traffic_bytes"], src
    return None, (f"null: no PMC profile of this exact launch shape in profiles/pmc_traffic.json "
                  f"(algorithmic bytes {alg_bytes / 1e9:.2f} GB)")


def blocks_per_eval(n_bytes: int, lam: int) -> int:
    """The reference's AES-256 block count per eval: 2 per level at LAMBDA = 16,
    4 per level at LAMBDA >= 32 (prg.rs:48-53 called once per level, lib.rs:176)."""
    return (2 if lam == 16 else 4) * 8 * n_bytes


HBM_WRITE_BPS = 8.0e12  # MI355X_MICROARCH.md HBM peak (a sequential fill measures 6.9 TB/s, scripts/hbm_write_bw.py)


def wide_roofline(m, nb, lam, kern_s, exec_bpe, bpe, kernel, engine):
    """LAMBDA >= 32 (C4): head and tail run back to back, so the bound is the sum of the
    head's AES time at the T-table LDS peak and the output's HBM write time."""
    t_aes = m * exec_bpe / PEAK_TT_BLOCKS
    t_out = m * lam / HBM_WRITE_BPS
    peak = m / (t_aes + t_out)
    achieved = m / kern_s
    return {"bound": "lds+hbm", "kernel": kernel, "engine": engine, "achieved": achieved / 1e6,
            "peak": peak / 1e6, "unit": "M evals/s", "frac": achieved / peak, "traffic": None,
            "algorithmic_bytes": m * (nb + lam), "kernel_ms": kern_s * 1e3, "hbm_GBps": m * (nb + lam) / kern_s / 1e9,
            "executed_blocks_per_eval": exec_bpe, "reference_blocks_per_eval": bpe,
            "aes_blocks_per_s_executed": m * exec_bpe / kern_s,
            "note": "peak = 1 / (executed AES-256 blocks per eval / 87.8 G blocks/s (T-table LDS bound) + "
                    "LAMBDA bytes per eval / 8 TB/s HBM write): the head (AES walk over bytes [0,32)) and the tail "
                    "(GF(2) combination writing bytes [32, LAMBDA)) run back to back"}


def lds_clock_bound(workload: str, kern_s: float):
    """Counter-backed bound of the workload's kernels from a committed profile
    (profiles/lds_clock_bound.json, scripts/lds_clock_bound.py): each kernel's LDS-array cycles per
    CU at the clock that kernel ran at, summed over one dispatch of each; frac = that bound / the
    same kernels' traced time in the profiled run.  None when no profile of the workload is committed."""
    try:
        with open(os.path.join(ROOT, "profiles", "lds_clock_bound.json")) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    for e in t:
        if e.get("workload") == workload:
            # frac within the profiled run (its clocks and its kernel times): a bound at one run's clocks
            # against another run's time would mix boxes
            return {"bound_ms": e["bound_ms"], "frac": e["frac_of_kernels"], "profiled_kernels_ms": e["kernels_ms"],
                    "this_run_kernel_ms": kern_s * 1e3,
                    "bound_ms_at_2p4ghz": e["bound_ms_at_2p4ghz"],
                    "clocks_ghz": {r["kernel"].split("<")[0]: round(r["clock_ghz"], 3) for r in e["kernels"]
                                   if "clock_ghz" in r},
                    "source": e["source"] + " via profiles/lds_clock_bound.json",
                    "note": "sum over the step's kernels of SQ_LDS_IDX_ACTIVE / 256 CUs / (the kernel's clock = "
                            "GRBM_GUI_ACTIVE / 8 XCDs / its mean duration): the LDS array 100 % busy at the clock "
                            "the chip held (DESIGN.md section 7), against the same kernels' traced time in that run (one dispatch "
                            "each: C5's step runs the eval kernels twice); bound_ms_at_2p4ghz: the same cycles at 2.4 GHz; "
                            "from a committed profile of this launch shape, not this run"}
    return None


def zero_bits(xs: torch.Tensor, skip_bits: int = 0) -> int:
    """Number of 0 bits in the points = left steps = the A blocks the stream engine
    encrypts on top of one B block per level (kernels_stream.h), not counting each
    point's first `skip_bits` (Msb0) bits: the levels a shared-prefix table covers."""
    lut = torch.tensor([8 - bin(i).count("1") for i in range(256)], dtype=torch.int32, device=xs.device)
    x2 = xs.reshape(xs.shape[0], -1)
    full, part = skip_bits // 8, skip_bits % 8
    tot = 0
    for off in range(0, x2.shape[0], 1 << 22):
        c = x2[off:off + (1 << 22)].to(torch.int64)
        tot += int(lut[c[:, full:]].sum().item())
        if part:  # the partial byte's first `part` bits are covered by the prefix
            tot -= int(lut[c[:, full] >> (8 - part)].sum().item()) - (8 - part) * c.shape[0]
    return tot


def dist_setup(n_gpus: int, backend: str = "nccl", force: bool = False):
    """One process per GPU.  A process group comes up for WORLD_SIZE > 1, and also at world
    size 1 with `force` (--force-dist): then the key broadcast, the per-rank all_gather_object
    and the timing all-reduce run through the backend (RCCL for nccl) exactly as at N > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    if world > 1 or force:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        # one rank per GPU; with --dist-backend gloo several ranks may share a device (a
        # rehearsal of the multi-rank path on a one-GPU box)
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, cmd, env=None, poll_s: float = 0.2) -> int:
    """`--gpus N` (N > 1) without a launcher (WORLD_SIZE unset): start N fresh rank processes
    running `cmd` with the environment torch.distributed.run would give them (RANK, LOCAL_RANK,
    WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1, a free MASTER_PORT), one per GPU
    (each rank takes device = LOCAL_RANK in dist_setup), and wait for them.  This process never
    touches the GPU and replaces itself with nothing: the ranks are children (fork + exec of a
    process with no HIP state).  Rank 0's stdout is this process's stdout, so the one JSON line
    reaches the caller unchanged.  When a rank fails, the others are ended (their own PIDs) and
    the exit status is the first failure's (128 + signal for a killed rank)."""
    base = dict(os.environ if env is None else env)
    port = str(_free_port())
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR=base.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen(list(cmd), env=e))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in live:
                    q.terminate()
        if live:
            time.sleep(poll_s)
    return rc


def pg() -> bool:
    """A process group is up (N > 1, or N = 1 with --force-dist)."""
    return dist.is_initialized()


def make_key(d: dcf_amd.DcfImpl, n_bytes: int, lam: int, world: int, seed: int, timing: dict = None):
    """Rank 0 runs gen on its GPU; the CWB and both seeds go to every rank by RCCL broadcast
    (its time, between two barriers and outside any timed region, goes into timing['key_broadcast_ms'])."""
    dev = torch.device("cuda", torch.cuda.current_device())
    rng = np.random.default_rng(seed)
    alpha, beta, s0, s1 = rng.bytes(n_bytes), rng.bytes(lam), rng.bytes(lam), rng.bytes(lam)
    cwb = torch.empty(dcf_amd.cwb_bytes(n_bytes, lam, 1), dtype=torch.uint8, device=dev)
    seeds = torch.empty((2, lam), dtype=torch.uint8, device=dev)
    if not pg() or dist.get_rank() == 0:
        k = d.gen(dcf_amd.CmpFn(alpha, beta), [s0, s1], dcf_amd.BoundState.LtBeta)
        cwb.copy_(torch.from_numpy(np.frombuffer(dcf_amd.share_to_cwb(k, n_bytes, lam), np.uint8).copy()))
        seeds.copy_(torch.from_numpy(np.frombuffer(s0 + s1, np.uint8).reshape(2, lam).copy()))
    torch.cuda.synchronize()
    if pg():
        dist.barrier()
    t0 = time.perf_counter()
    broadcast_key([cwb, seeds], src=0)
    torch.cuda.synchronize()
    if timing is not None:
        timing["key_broadcast_ms"] = (time.perf_counter() - t0) * 1e3
        timing["key_bytes"] = cwb.numel() + seeds.numel()
    return cwb, seeds, alpha, beta


def gen_points(m: int, n_bytes: int, start: int, seed: int) -> torch.Tensor:
    """Global points [start, start + m) (the rank's slice), drawn on device from a
    generator keyed by (seed, slice start)."""
    g = torch.Generator(device="cuda")
    g.manual_seed(seed * 1000003 + start)
    return torch.randint(0, 256, (m, n_bytes), dtype=torch.uint8, device="cuda", generator=g)


def oracle_key(cwb_h: bytes, n_bytes: int, lam: int, K: int = 1, key: int = 0):
    """Key `key` of a K-key CWB (include/dcf_hip.h layout) for the oracle (checker only)."""
    from oracle import oracle as O
    n = 8 * n_bytes
    c = np.frombuffer(cwb_h, np.uint8)
    k = O.OracleKey(n_bytes, lam)
    k.cw_s[:] = c[:n * K * lam].reshape(n, K, lam)[:, key]
    k.cw_v[:] = c[n * K * lam:2 * n * K * lam].reshape(n, K, lam)[:, key]
    k.cw_t[:] = c[2 * n * K * lam:2 * n * K * lam + n * K].reshape(n, K)[:, key]
    off = dcf_amd.cwb_np1_offset(n_bytes, lam, K)
    k.cw_np1[:] = c[off:off + K * lam].reshape(K, lam)[key]
    return k


def host_threads() -> int:
    return max(1, min(16, len(os.sched_getaffinity(0))))  # the GPU box's CPU share is 16


def cpu_baseline(keys, n_bytes, lam, cwb_h: bytes, seeds, xs_sample: np.ndarray, ys_gpu, target_s: float,
                 prg_kind: str = "hirose", threads: int = 0, parties=(0,)):
    """Time the C restatement of the reference eval (oracle/dcf_oracle.c: AES-NI, one
    pthread per core over contiguous point chunks like rayon, lib.rs:194-199) on this
    host, on a bounded sample: calibrate on a small slice, then run ~target_s of CPU
    work (whole-sample repeats when the sample is smaller than that).  ys_gpu[b]: the
    GPU's outputs of party b for the sample rows (the check, `matches_gpu`)."""
    from oracle import oracle as O
    threads = threads or host_threads()
    P = (O.OracleMmoPrg if prg_kind == "mmo" else O.OraclePrg)(keys, lam)
    k = oracle_key(cwb_h, n_bytes, lam)
    cal = xs_sample[: min(len(xs_sample), max(threads, 8192 * threads * 16 // lam))]
    t0 = time.perf_counter()
    matches = True
    for b in parties:
        y = O.eval_(P, b, k, seeds[b], cal, nthreads=threads)
        matches = matches and bool(np.array_equal(y, ys_gpu[b][: len(cal)]))
    dt = time.perf_counter() - t0
    rate = len(cal) * len(parties) / dt
    m = int(min(len(xs_sample), max(len(cal), rate * target_s / len(parties))))
    reps = max(1, min(200, int(round(rate * target_s / (m * len(parties))))))
    t0 = time.perf_counter()
    for r in range(reps):
        for b in parties:
            y = O.eval_(P, b, k, seeds[b], xs_sample[:m], nthreads=threads)
            if r == 0:
                matches = matches and bool(np.array_equal(y, ys_gpu[b][:m]))
    dt = time.perf_counter() - t0
    who = "both parties" if len(parties) == 2 else f"party {parties[0]}"
    return {
        "value": m * len(parties) * reps / dt, "unit": "evals/s", "cores": threads, "kind": "port",
        "sample": f"{m} of the GPU's points (first rows of rank 0's slice) x {reps} repeat(s), {who}, same key; "
                  f"C restatement of lib.rs:163-204 + prg.rs:42-73 with AES-NI, {threads} thread(s); {dt:.1f} s",
        "ms_per_batch": dt / reps * 1e3, "aesni": P.uses_aesni, "matches_gpu": matches,
    }


def timed_loop(step, steps: int, warmup: int, world: int, stream=None, local: dict = None):
    """Run `warmup` untimed steps, then time `steps` steps bracketed by barrier + sync.
    Returns (wall seconds, max over ranks; seconds per step on `stream` by HIP events).
    local (optional) receives this rank's own wall seconds and event seconds per step."""
    stream = stream or torch.cuda.current_stream()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if pg():
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if pg():
        dist.barrier()
    torch.cuda.synchronize()
    w = time.perf_counter() - t0
    k = ev0.elapsed_time(ev1) / 1e3 / steps
    if local is not None:
        local.update(wall_s=w, event_s_per_step=k)
    t = torch.tensor([w], dtype=torch.float64, device="cuda")
    if pg():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), k


def gather_per_rank(world: int, rec: dict):
    """Every rank's measurement record on rank 0 (all_gather_object: small host objects, outside
    the timed region); [rec] at N = 1."""
    if not pg():
        return [rec]
    out = [None] * world
    dist.all_gather_object(out, rec)
    return out


def per_rank_summary(recs, steps: int):
    """The N > 1 line's per-rank block: kernel / wall time per rank and the imbalance that a
    scaling curve would hide (max over min of the ranks' step times)."""
    walls = [r["wall_s"] / steps * 1e3 for r in recs]
    kern = [r["kernel_ms"] for r in recs]
    return {"ranks": recs, "wall_ms_per_step_min": min(walls), "wall_ms_per_step_max": max(walls),
            "kernel_ms_min": min(kern), "kernel_ms_max": max(kern),
            "imbalance": max(walls) / min(walls) if min(walls) > 0 else None,
            "note": "per rank: its own wall and HIP-event time per step (the line's value uses the max over "
                    "ranks), one extra untimed eval with phase events (table_ms = shared-prefix table / digest "
                    "build, walk_ms = walk kernels) and the prefix depth its slice used"}


def host_path(d, k_share_fn, xs_dev, lam, parties: int, steps: int):
    """`dcf_eval` on host buffers (what a Rust DcfHip::eval pays: PCIe both ways through
    the pipelined staging path), over the same points; evals/s including PCIe."""
    xs_h = xs_dev.cpu().numpy()
    m = xs_h.shape[0]
    ys = [np.empty((m, lam), np.uint8) for _ in range(parties)]
    shares = [k_share_fn(b) for b in range(parties)]
    for b in range(parties):  # warm-up: allocates the pooled staging buffers
        d.eval(bool(b), shares[b], xs_h, ys[b])
    t0 = time.perf_counter()
    for _ in range(steps):
        for b in range(parties):
            d.eval(bool(b), shares[b], xs_h, ys[b])
    dt = time.perf_counter() - t0
    return {"value": m * parties * steps / dt, "unit": "evals/s", "ms_per_step": dt / steps * 1e3,
            "pcie_bytes_per_step": parties * m * (xs_h.shape[1] + lam),
            "note": "dcf_eval (host buffers, synchronous): x H2D + y D2H through pinned staging, 3 streams, "
                    "128 MiB chunks overlapping copies with kernels; includes the host memcpy to/from staging"}, ys


def run_eval(args, world, rank):
    nb, lam = args.n_bytes, args.lam
    if args.scaling == "strong":
        start, m = point_slice(args.points, world, rank)
        global_points = args.points
    else:
        start, m = weak_slice(args.points, rank)
        global_points = args.points * world
    rng = np.random.default_rng(0xDCF0001)
    # benches/dcf_batch_eval.rs:7 uses 2 AES keys at LAMBDA = 16; benches/dcf_large_lambda.rs:10 uses 2048.
    if args.prg == "mmo":  # Aes128MatyasMeyerOseasPrg (north_star's PRG; not in the reference): 4 AES-128 keys
        keys = [rng.bytes(16) for _ in range(4 * lam // 16)]  # per output and 16-byte block
        prg = dcf_amd.Aes128MatyasMeyerOseasPrg(keys, lam, device=torch.cuda.current_device())
    else:
        keys = [rng.bytes(32) for _ in range(2 if lam == 16 else 2048)]
        prg = dcf_amd.Aes256HirosePrg(keys, lam, device=torch.cuda.current_device())
    prg.set_eval_mode(args.eval_mode)
    prg.set_prefix_levels(args.prefix)
    pfx = prg.eval_prefix_levels(nb, 1, m)  # shared-prefix depth this eval uses (0 = none)
    d = dcf_amd.DcfImpl(nb, lam, prg)
    ktime = {}
    cwb, seeds, alpha, beta = make_key(d, nb, lam, world, 0xDCF0002, ktime)
    s0 = seeds[0].contiguous()
    s1 = seeds[1].contiguous()
    xs = gen_points(m, nb, start, 0xDCF0003)
    ys = torch.empty((m, lam), dtype=torch.uint8, device="cuda")
    # C1 (benches/dcf_batch_eval.rs shape) evaluates both parties per step.
    parties = 2 if args.workload == "c1" else 1
    ys1 = torch.empty_like(ys) if parties == 2 else None

    def step():
        d.eval_device(False, cwb, s0, xs, ys)
        if parties == 2:
            d.eval_device(True, cwb, s1, xs, ys1)

    mine = {}
    wall, kern_s = timed_loop(step, args.steps, args.warmup, world, local=mine)
    kern_s /= parties
    dev_blocks = prg.last_eval_blocks()  # stream engine: AES blocks of the last launch, counted on the device
    # one more (untimed) eval with phase events: this rank's table build vs walk split
    prg.set_phase_timing(True)
    d.eval_device(False, cwb, s0, xs, ys)
    torch.cuda.synchronize()
    table_ms, walk_ms, depth = prg.last_eval_phases()
    prg.set_phase_timing(False)
    rank_rec = {"rank": rank, "device": torch.cuda.current_device(), "points": m, "start": start,
                "wall_s": mine["wall_s"], "kernel_ms": kern_s * 1e3, "table_ms": table_ms, "walk_ms": walk_ms,
                "prefix_levels": depth, "key_broadcast_ms": ktime.get("key_broadcast_ms")}
    per_rank = gather_per_rank(world, rank_rec)
    no_prefix = None
    if pfx and not args.no_compare:
        # the same batch without the shared-prefix table (each point walks all 8N levels)
        prg.set_prefix_levels(0)
        w0, k0 = timed_loop(step, args.steps, args.warmup, world)
        np_blocks = prg.last_eval_blocks()
        prg.set_prefix_levels(args.prefix)
        small_path = args.eval_mode == 0 and lam == 16 and m < CUS * 1024 * 2  # the pair walk: A and B every level
        no_prefix = {"value": global_points * args.steps * parties / w0, "kernel_ms": k0 / parties * 1e3,
                     "executed_blocks_per_eval": 16 * nb if args.prg == "mmo" else 2 * 8 * nb if small_path else (
                         np_blocks / m if np_blocks else 8 * nb + zero_bits(xs) / m),
                     "speedup": w0 / wall}
    total_evals = global_points * args.steps * parties
    value = total_evals / wall
    check = slice_check(d, cwb, s0, ys, nb, lam, args, world, rank) if args.check else None
    abi_check = None
    if rank == 0 and (world > 1 or args.abi_check):
        prg_cls = dcf_amd.Aes128MatyasMeyerOseasPrg if args.prg == "mmo" else dcf_amd.Aes256HirosePrg
        abi_check = multi_gpu_abi_check(keys, nb, lam, prg_cls, d, cwb, s0,
                                        points=min(1 << 20, max(1, (1 << 30) // (lam * 8))))
    bpe = blocks_per_eval(nb, lam)
    if args.prg == "mmo" and lam > 16:
        bpe = 4 * 8 * nb * (lam // 16)  # the MMO PRG's full output per level: 4 outputs x LAMBDA/16 blocks
    engine = ENGINE[args.eval_mode] if lam == 16 else "ttable"
    if args.prg == "mmo":
        engine = "mmo"
    elif args.eval_mode == 0 and lam == 16 and m < CUS * 1024 * 2:
        engine = "ttable-small"  # auto mode's small-batch path: lockstep walk (dcf_hip.hip eval_launch)
    # Blocks the dominant kernel actually encrypts per eval: the reference count, except the
    # stream engine, which encrypts B on every level and A on left (x bit 0) levels only.
    # With a shared-prefix table of depth D a point walks levels D..8N-1 only, and the
    # table costs 2 blocks per node of the top tree (2^(D+1) - 2), spread over the batch.
    # MMO: 2 AES-128 blocks per level below the prefix (the table: 2 per node as well).
    if engine == "stream":
        # B every level + A on left levels, minus the B blocks reused after a right step at
        # t = 0 (kernels_stream.h): counted by the kernel itself, plus the prefix table
        walk = dev_blocks / m if dev_blocks else (8 * nb - pfx) + zero_bits(xs, pfx) / m
        exec_bpe = walk + (2 ** (pfx + 1) - 2) / m
    elif engine == "mmo" or (engine == "ttable-small" and pfx):
        # lockstep walks (A and B every level) below a shared prefix (auto on the small path since r06)
        exec_bpe = 2 * (8 * nb - pfx) + (2 ** (pfx + 1) - 2) / m
    else:
        exec_bpe = bpe
    if lam > 16 and args.prg == "mmo":
        # multi-block MMO: the side's s and v blocks for every 16-byte block, every level
        engine = "mmo-wide"
        exec_bpe = 2 * 8 * nb * (lam // 16)
    elif lam > 16:
        # LAMBDA >= 32: the stream head encrypts B, A (left) or B, D, C (right) per level, and the
        # tail writes LAMBDA - 32 output bytes per eval: time bound = AES (LDS) + output (HBM write).
        engine = "stream-head"
        if engine == "stream-head":
            # below a shared prefix of pfx levels (k_wpfx_build: 4 blocks per parent node); the
            # walk's blocks are counted by the kernel (B reuse after a right step at t = 0 skips
            # some B blocks, kernels_wide_stream.h), else 2 per left and 3 per right level
            walk = dev_blocks / m if dev_blocks else 3 * (8 * nb - pfx) - zero_bits(xs, pfx) / m
            exec_bpe = walk + 4 * (2 ** pfx - 1) / m
    per_gpu_blocks = m * exec_bpe / kern_s
    # HBM bytes per launch of the dominant kernel: x in, y out, and with a shared prefix
    # one 32-byte table row gathered per point (kernels16.h PrefixTable)
    alg_bytes = m * (nb + lam) + (m * 32 if pfx else 0)
    kernel = KERNEL.get(engine, "k_eval16") if lam == 16 else (
        "k_mmo_wide_eval" if engine == "mmo-wide" else
        "k_eval_wide_head_stream+k_eval_wide_tail" if engine == "stream-head" else "k_eval_wide_head+k_eval_wide_tail")
    peak = engine_peak(engine)
    traffic, traffic_src = traffic_fields(kernel, m, nb, lam, pfx, alg_bytes)
    slicing = (f"2^{int(np.log2(args.points))} points split over {world} GPU(s) (strong)" if args.scaling == "strong"
               else f"{m} points per GPU (weak)")
    out = {
        "metric": METRIC, "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"{args.workload.upper()}: N={nb} ({8 * nb}-bit x), lambda={lam}, "
                               f"{'Aes128MatyasMeyerOseasPrg' if args.prg == 'mmo' else 'Aes256HirosePrg'} "
                               f"({len(keys)} AES keys), 1 key, {slicing}, in HBM, "
                               f"{'both parties' if parties == 2 else 'party 0'}, eval only",
                   "n_bytes": nb, "lambda": lam, "points_per_gpu": m, "global_points": global_points,
                   "parallelism": f"points sharded over {world} GPU(s) in contiguous slices, "
                                  "no collective in timed region"},
        "aes_blocks_per_s_reference_count": value * bpe,
        "aes_blocks_per_s_executed": value * exec_bpe,
        "roofline": wide_roofline(m, nb, lam, kern_s, exec_bpe, bpe, kernel, engine) if (lam > 16 and engine != "mmo-wide") else {
            "bound": "lds",
            "kernel": kernel, "engine": engine,
            "achieved": per_gpu_blocks / 1e9, "peak": peak / 1e9, "unit": "G AES-128 blocks/s" if engine.startswith("mmo") else "G AES-256 blocks/s",
            "frac": per_gpu_blocks / peak, "traffic": traffic, "traffic_source": traffic_src,
            "algorithmic_bytes": alg_bytes, "kernel_ms": kern_s * 1e3,
            "hbm_GBps": alg_bytes / kern_s / 1e9,
            "ttable_only_peak": PEAK_TT_BLOCKS / 1e9,
            "measured_ceiling": None if engine.startswith("mmo") else measured_ceiling(per_gpu_blocks),
            "executed_blocks_per_eval": exec_bpe, "reference_blocks_per_eval": bpe,
            "prefix_levels": pfx, "no_prefix": no_prefix,
            "note": "achieved = AES blocks the kernel encrypts per second (stream engine: B every "
                    "level + A on left levels, minus B blocks reused after a right step at t = 0, counted on the device; mmo: 2 AES-128 per level; both below a shared-prefix table "
                    "of prefix_levels levels built inside the timed call and counted; other engines: the "
                    "reference count, 2 per level); "
                    "aes_blocks_per_s_reference_count above uses the reference count (2 per level; the kernels skip "
                    "unused A blocks, reused B blocks and the shared prefix, so it exceeds the LDS peak), "
                    "aes_blocks_per_s_executed the blocks actually encrypted.  Peak per GPU at 2.4 GHz: T-table "
                    "engines LDS-bound (32 ds_read_b32 lookups/clk/CU, 224 per block; DESIGN.md section 4)",
        },
    }
    if lam > 16 and engine != "mmo-wide":
        out["roofline"]["prefix_levels"] = pfx  # wide stream head below a shared-prefix table
        if args.workload == "c4" and nb == 16 and m == 1 << 22:
            out["roofline"]["lds_clock_bound"] = lds_clock_bound("C4", kern_s)
    elif args.prg == "hirose" and (args.workload, nb, m) in (("c1", 16, 100_000), ("c2", 4, 1 << 24), ("c3", 16, 1 << 28)):
        # the default launch shapes the committed profiles ran (per-party kernel time)
        out["roofline"]["lds_clock_bound"] = lds_clock_bound(args.workload.upper(), kern_s)
        out["roofline"]["traffic"], out["roofline"]["traffic_source"] = traffic_fields(
            kernel, m, nb, lam, pfx, m * (nb + lam))
    if check is not None:
        out["slice_check"] = check
    if abi_check is not None:
        out["multi_gpu_abi_check"] = abi_check
    out["phases"] = {"table_ms": table_ms, "walk_ms": walk_ms, "prefix_levels": depth,
                     "note": "rank 0, one untimed eval with phase events (dcf_prg_set_phase_timing)"}
    if pg():
        out["per_rank"] = per_rank_summary(per_rank, args.steps)
        out["key_broadcast"] = {"ms": ktime.get("key_broadcast_ms"), "bytes": ktime.get("key_bytes"),
                                "backend": args.dist_backend, "note": "once, before timing (outside the timed region)"}
    host_ys = None
    if args.host_path or args.workload == "c1":
        share = dcf_amd.cwb_to_share(cwb.cpu().numpy().tobytes(), nb, lam, [])
        sd = seeds.cpu().numpy()
        out["host_path"], host_ys = host_path(
            d, lambda b: dcf_amd.Share([sd[b].tobytes()], share.cws, share.cw_np1), xs, lam, parties,
            max(1, min(args.steps, 3)))
        out["host_path"]["matches_device_path"] = bool(np.array_equal(host_ys[0], ys.cpu().numpy()))
    if rank == 0 and world == 1 and not args.no_cpu:  # cpu_baseline: rank 0 at N=1 only
        ns = min(m, 1 << 26, max(4096, (1 << 30) // lam))  # at most ~1 GiB of outputs copied back
        xs_h = xs[:ns].cpu().numpy()
        ys_h = [ys[:ns].cpu().numpy()] + ([ys1[:ns].cpu().numpy()] if parties == 2 else [])
        cwb_h = cwb.cpu().numpy().tobytes()
        sd = [bytes(seeds[0].cpu().numpy().tobytes()), bytes(seeds[1].cpu().numpy().tobytes())]
        pp = tuple(range(parties))
        out["cpu_baseline"] = cpu_baseline(keys, nb, lam, cwb_h, sd, xs_h, ys_h, args.cpu_seconds, args.prg,
                                           parties=pp)
        if args.workload == "c1":  # all cores and 1 core
            out["cpu_baseline_1core"] = cpu_baseline(keys, nb, lam, cwb_h, sd, xs_h, ys_h, args.cpu_seconds / 2,
                                                     args.prg, threads=1, parties=pp)
    return out


def ys_digest(ys: torch.Tensor) -> int:
    """Order-sensitive 64-bit digest of an output slice (row-weighted byte sums), in chunks of
    rows so the int64 temporaries stay small."""
    c = torch.arange(1, ys.shape[1] + 1, device=ys.device, dtype=torch.int64)
    tot = torch.zeros((), dtype=torch.int64, device=ys.device)
    step = max(1, (1 << 24) // max(1, ys.shape[1]))
    for off in range(0, ys.shape[0], step):
        y = ys[off:off + step].to(torch.int64)
        w = torch.arange(off + 1, off + y.shape[0] + 1, device=ys.device, dtype=torch.int64).unsqueeze(1)
        tot += (y * w).sum() + (y.sum(0) * c).sum()
    return int(tot.item())


def slice_check(d, cwb, s0, ys, nb, lam, args, world, rank):
    """Multi-rank self-check: every rank's output digest goes to rank 0, which regenerates each
    rank's slice of points, evaluates it itself and compares."""
    digs = [ys_digest(ys)]
    if pg():  # all_gather_object: gloo's all_gather takes host tensors only
        digs = [None] * world
        dist.all_gather_object(digs, ys_digest(ys))
    if rank != 0:
        return None
    ok = []
    for r in range(world):
        st, cnt = (point_slice(args.points, world, r) if args.scaling == "strong" else weak_slice(args.points, r))
        xr = gen_points(cnt, nb, st, 0xDCF0003)
        yr = d.eval_device(False, cwb, s0, xr)
        torch.cuda.synchronize()
        ok.append(ys_digest(yr) == int(digs[r]))
    return {"ranks": world, "slices_match": all(ok), "per_rank": ok}


def multi_gpu_abi_check(keys, nb, lam, prg_cls, d, cwb, s0, points: int = 1 << 20):
    """N > 1, rank 0, after timing: one dcf_eval_multi_gpu_device call (the one-process
    multi-GPU C ABI) over every visible device (at least 2 prgs: on a one-GPU box both sit on
    device 0), slices gathered into one buffer on device 0 — hipMemcpyPeerAsync over xGMI for
    every slice on another device — and compared byte for byte with rank 0's own
    dcf_eval_device over the same points.  Never raises: a failure is recorded in the line."""
    t0 = time.perf_counter()
    ndev = torch.cuda.device_count()
    G = max(2, min(ndev, 8))
    devs = [g % ndev for g in range(G)]
    rec = {"devices": devs, "points": points, "peer_slices": sum(1 for v in devs if v != devs[0])}
    try:
        impls = [dcf_amd.DcfImpl(nb, lam, prg_cls(keys, lam, device=v)) for v in devs]
        mg = dcf_amd.MultiGpuDcf(impls)
        xs = gen_points(points, nb, 0, 0xDCF0004)
        slices = []
        for g, v in enumerate(devs):
            st, cnt = dcf_amd.point_slice(points, G, g)
            slices.append(xs[st:st + cnt].to(torch.device("cuda", v)).contiguous())
        gather = torch.empty((points, lam), dtype=torch.uint8, device=xs.device)
        cwb_h = cwb.cpu().numpy().tobytes()
        ys_sl = mg.eval_device(False, cwb_h, s0.cpu().numpy().tobytes(), slices, gather=gather)
        ref = d.eval_device(False, cwb, s0, xs)
        torch.cuda.synchronize()
        rows = [dcf_amd.point_slice(points, G, g) for g in range(G)]
        rec["slices_match"] = all(torch.equal(ys_sl[g].to(xs.device), ref[st:st + c]) for g, (st, c) in enumerate(rows))
        rec["gather_matches"] = bool(torch.equal(gather, ref))
        rec["ok"] = rec["slices_match"] and rec["gather_matches"]
    except Exception as e:  # noqa: BLE001 — recorded, the line still prints
        rec["ok"] = False
        rec["error"] = f"{type(e).__name__}: {e}"
    rec["ms"] = (time.perf_counter() - t0) * 1e3
    rec["note"] = ("dcf_eval_multi_gpu_device over the devices listed (prgs from the same keys), gather on device "
                   "0; peer_slices = slices copied from another device (hipMemcpyPeerAsync, dcf_hip.hip); compared "
                   "with dcf_eval_device on rank 0; untimed, after the timed region")
    return rec


def c5_inputs(K: int, kstart: int, nb: int, lam: int, P: int):
    """C5 keys [kstart, kstart + K): alpha, beta, both root seeds and P points per key, drawn on
    device from a generator keyed by the slice start (any rank can regenerate any slice)."""
    g = torch.Generator(device="cuda")
    g.manual_seed(5 * 1000003 + kstart)
    rnd = lambda *s: torch.randint(0, 256, s, dtype=torch.uint8, device="cuda", generator=g)  # noqa: E731
    alpha, beta, s0, s1 = rnd(K, nb), rnd(K, lam), rnd(K, lam), rnd(K, lam)
    return alpha, beta, s0, s1, rnd(K * P, nb)


def c5_check(d, cwb, y0, y1, args, world, rank, nb, lam, P):
    """Multi-rank self-check of C5: every rank's (CWB, party-0 and party-1 outputs) digests go
    to rank 0, which regenerates each rank's keys and points, runs batched gen and both
    parties' multi-key eval itself, and compares."""
    mine = [ys_digest(cwb.view(-1, 16)), ys_digest(y0), ys_digest(y1)]
    digs = [mine]
    if pg():
        digs = [None] * world
        dist.all_gather_object(digs, mine)
    if rank != 0:
        return None
    ok = []
    for r in range(world):
        st, K = (point_slice(args.keys, world, r) if args.scaling == "strong" else weak_slice(args.keys, r))
        alpha, beta, s0, s1, xs = c5_inputs(K, st, nb, lam, P)
        cw = d.gen_batch_device(alpha, beta, s0, s1, dcf_amd.BoundState.LtBeta,
                                torch.zeros(dcf_amd.cwb_bytes(nb, lam, K), dtype=torch.uint8, device="cuda"))
        a = d.eval_multikey_device(False, cw, s0, xs, P)
        b = d.eval_multikey_device(True, cw, s1, xs, P)
        torch.cuda.synchronize()
        ok.append([ys_digest(cw.view(-1, 16)), ys_digest(a), ys_digest(b)] == [int(v) for v in digs[r]])
    return {"ranks": world, "slices_match": all(ok), "per_rank": ok}


def run_c5(args, world, rank):
    """C5: K independent keys x 64 points: batched gen + eval of both parties per step.
    Strong scaling by default: the 2^20 keys are split over the ranks (dcf_point_slice)."""
    nb, lam, P = args.n_bytes, 16, 64
    if args.scaling == "strong":
        kstart, K = point_slice(args.keys, world, rank)
        global_keys = args.keys
    else:
        kstart, K = weak_slice(args.keys, rank)
        global_keys = args.keys * world
    rng = np.random.default_rng(0xDCF0005)
    keys = [rng.bytes(32) for _ in range(2)]
    prg = dcf_amd.Aes256HirosePrg(keys, lam, device=torch.cuda.current_device())
    d = dcf_amd.DcfImpl(nb, lam, prg)
    alpha, beta, s0, s1, xs = c5_inputs(K, kstart, nb, lam, P)
    # zeroed: gen writes every key byte, the padding before cw_np1 stays 0 (c5_check digests it all)
    cwb = torch.zeros(dcf_amd.cwb_bytes(nb, lam, K), dtype=torch.uint8, device="cuda")
    y0 = torch.empty((K * P, lam), dtype=torch.uint8, device="cuda")
    y1 = torch.empty_like(y0)
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    phase = [0.0, 0.0, 0.0]

    def step(record=False):
        if record:
            ev[0].record(stream)
        d.gen_batch_device(alpha, beta, s0, s1, dcf_amd.BoundState.LtBeta, cwb)
        if record:
            ev[1].record(stream)
        d.eval_multikey_device(False, cwb, s0, xs, P, y0)
        if record:
            ev[2].record(stream)
        d.eval_multikey_device(True, cwb, s1, xs, P, y1)
        if record:
            ev[3].record(stream)

    # block counts on the device: party 0's eval alone, then party 1's (the last launch)
    d.gen_batch_device(alpha, beta, s0, s1, dcf_amd.BoundState.LtBeta, cwb)
    d.eval_multikey_device(False, cwb, s0, xs, P, y0)
    torch.cuda.synchronize()
    b0 = prg.last_eval_blocks()
    mine = {}
    wall, step_s = timed_loop(step, args.steps, args.warmup, world, local=mine)
    b1 = prg.last_eval_blocks()
    # per-phase HIP-event times over the same number of steps (separate loop: events between phases)
    for _ in range(args.steps):
        step(record=True)
        torch.cuda.synchronize()
        for i in range(3):
            phase[i] += ev[i].elapsed_time(ev[i + 1]) / 1e3 / args.steps
    evals = 2 * global_keys * P * args.steps
    gen_blocks = 4 * 8 * nb * K                  # k_gen16: A and B of both parties' PRG per level
    eval_blocks = b0 + b1                        # multi-key stream engine, counted on the device
    n = 8 * nb
    cwb_b = dcf_amd.cwb_bytes(nb, lam, K)
    dig_b = K * n * 33                           # key-major digest (k_cw_keymajor): 32 B CW + 1 B t per level
    key_bytes = cwb_b + 2 * (cwb_b + 2 * dig_b)  # gen writes CWB; per eval: digest reads CWB, writes + reads digest
    io_bytes = K * (nb + 3 * lam) + 2 * K * P * (nb + lam)
    alg_bytes = key_bytes + io_bytes
    peak = PEAK_TT_BLOCKS
    achieved = (gen_blocks + eval_blocks) / step_s
    eval_s = phase[1] + phase[2]
    traffic, traffic_src = traffic_fields("k_gen16+2*k_mk_prefix16+2*k_cw_keymajor+2*k_eval16_stream", K * P, nb, lam, 0, alg_bytes)
    out = {"metric": "C5 batched gen + eval (both parties)", "value": evals / wall, "unit": "evals/s",
           "keys_per_s": global_keys * args.steps / wall, "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
           "scaling": args.scaling, "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "aes_blocks_per_s_reference_count": evals / wall * blocks_per_eval(nb, lam) + global_keys * args.steps / wall * 4 * n,
           "aes_blocks_per_s_executed_per_gpu": (gen_blocks + eval_blocks) / step_s,
           "config": {"workload": f"C5: {global_keys} keys x {P} points ({K} keys on this GPU), N={nb}, "
                                  f"lambda={lam}, batched gen + multi-key eval of both parties per step",
                      "n_bytes": nb, "lambda": lam, "keys_per_gpu": K, "points_per_key": P},
           "phases_ms": {"gen": phase[0] * 1e3, "eval_party0": phase[1] * 1e3, "eval_party1": phase[2] * 1e3,
                         "note": "HIP events on the launch stream; each eval includes its key-major CW digest "
                                 "(k_cw_keymajor) — profiles/ has the per-kernel split"},
           "key_traffic_GBps": key_bytes / step_s / 1e9,
           "roofline": {"bound": "lds", "kernel": "k_gen16 + k_mk_prefix16 + k_cw_keymajor + k_eval16_stream<MULTI> (whole step)",
                        "engine": "stream (multi-key)", "achieved": achieved / 1e9, "peak": peak / 1e9,
                        "unit": "G AES-256 blocks/s", "frac": achieved / peak,
                        "eval_only": {"achieved": eval_blocks / eval_s / 1e9, "frac": eval_blocks / eval_s / peak,
                                      "executed_blocks_per_eval": eval_blocks / (2 * K * P),
                                      "measured_ceiling": measured_ceiling(eval_blocks / eval_s)},
                        "gen_only": {"achieved": gen_blocks / phase[0] / 1e9, "frac": gen_blocks / phase[0] / peak},
                        "traffic": traffic, "traffic_source": traffic_src, "algorithmic_bytes": alg_bytes,
                        "lds_clock_bound": lds_clock_bound("C5", step_s) if (K, nb) == (1 << 20, 16) else None,
                        "kernel_ms": step_s * 1e3, "hbm_GBps": alg_bytes / step_s / 1e9,
                        "executed_blocks_per_step": gen_blocks + eval_blocks,
                        "note": "gen: 4 AES-256 blocks per level per key (k_gen16); eval: blocks the multi-key "
                                "stream engine encrypts, counted on the device (B every level, A on left levels, "
                                "minus reused B); peak = T-table LDS bound 87.8 G blocks/s"}}
    if pg():
        recs = gather_per_rank(world, {"rank": rank, "keys": K, "key_start": kstart, "wall_s": mine["wall_s"],
                                       "kernel_ms": step_s * 1e3, "gen_ms": phase[0] * 1e3,
                                       "eval_ms": (phase[1] + phase[2]) * 1e3})
        out["per_rank"] = per_rank_summary(recs, args.steps)
    if args.check:
        chk = c5_check(d, cwb, y0, y1, args, world, rank, nb, lam, P)
        if chk is not None:
            out["slice_check"] = chk
    if rank == 0 and world == 1 and not args.no_cpu:  # cpu_baseline: rank 0 at N=1 only
        out["cpu_baseline"] = c5_cpu_baseline(keys, nb, lam, alpha, beta, s0, s1, xs, cwb, y0, y1, K, P,
                                              args.cpu_seconds)
    return out


def c5_cpu_baseline(keys, nb, lam, alpha, beta, s0, s1, xs, cwb, y0, y1, K, P, target_s):
    """Oracle gen + eval of both parties for a bounded sample of C5's keys, keys spread over
    host threads (ctypes releases the GIL), checked against the GPU's CWB and outputs."""
    from oracle import oracle as O
    threads = host_threads()
    Po = O.OraclePrg(keys, lam)
    A, B, S0, S1 = (t.cpu().numpy() for t in (alpha, beta, s0, s1))
    cw = cwb.cpu().numpy().tobytes()

    def work(ids):
        ok_all = True
        for key in ids:
            ok = O.gen(Po, A[key].tobytes(), B[key].tobytes(), S0[key].tobytes(), S1[key].tobytes(), 0)
            xk = X[key * P:(key + 1) * P]
            ya = O.eval_(Po, 0, ok, S0[key].tobytes(), xk)
            yb = O.eval_(Po, 1, ok, S1[key].tobytes(), xk)
            if check:
                kk = oracle_key(cw, nb, lam, K, int(key))
                ok_all = ok_all and np.array_equal(kk.cw_s, ok.cw_s) and np.array_equal(kk.cw_v, ok.cw_v) \
                    and np.array_equal(ya, Y0[key * P:(key + 1) * P]) and np.array_equal(yb, Y1[key * P:(key + 1) * P])
        return ok_all

    def run(nkeys):
        ids = np.arange(nkeys)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(work, np.array_split(ids, threads)))
        return time.perf_counter() - t0, all(res)

    ncal = min(K, 64 * threads)
    X = xs[:ncal * P].cpu().numpy()
    Y0, Y1 = y0[:ncal * P].cpu().numpy(), y1[:ncal * P].cpu().numpy()
    check = True
    dt, ok = run(ncal)
    nk = int(min(K, max(ncal, ncal / dt * target_s)))
    X = xs[:nk * P].cpu().numpy()
    Y0, Y1 = y0[:nk * P].cpu().numpy(), y1[:nk * P].cpu().numpy()
    check = False
    dt, _ = run(nk)
    return {"value": 2 * nk * P / dt, "unit": "evals/s", "keys_per_s": nk / dt, "cores": threads, "kind": "port",
            "sample": f"gen + eval of both parties (64 points each) for the first {nk} keys, keys split over "
                      f"{threads} threads; C restatement of lib.rs:86-204 + prg.rs:42-73 with AES-NI; {dt:.1f} s",
            "matches_gpu": ok}


def run_fd(args, world, rank):
    """Full-domain eval: y for every x in [0, 2^(8N)), N = 4 by default
    (the 32-bit fixed-point shape: 2^32 outputs, 64 GiB), party 0, one key.  Ranks
    evaluate the same key (replicas: the tree expansion has no point slice to shard)."""
    nb, lam = args.n_bytes, 16
    rng = np.random.default_rng(0xDCF0001)
    mmo = args.prg == "mmo"
    if mmo:
        keys = [rng.bytes(16) for _ in range(4)]
        prg = dcf_amd.Aes128MatyasMeyerOseasPrg(keys, lam, device=torch.cuda.current_device())
    else:
        keys = [rng.bytes(32) for _ in range(2)]
        prg = dcf_amd.Aes256HirosePrg(keys, lam, device=torch.cuda.current_device())
    prg_name = "Aes128MatyasMeyerOseasPrg" if mmo else "Aes256HirosePrg"
    d = dcf_amd.DcfImpl(nb, lam, prg)
    cwb, seeds, alpha, beta = make_key(d, nb, lam, world, 0xDCF0002)
    s0 = seeds[0].contiguous()
    npts = 1 << (8 * nb)
    ys = torch.empty((npts, lam), dtype=torch.uint8, device="cuda")
    for _ in range(args.warmup):
        d.eval_full_domain_device(False, cwb, s0, ys)
    torch.cuda.synchronize()
    if pg():
        dist.barrier()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        d.eval_full_domain_device(False, cwb, s0, ys)
    ev1.record(stream)
    torch.cuda.synchronize()
    if pg():
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_s = ev0.elapsed_time(ev1) / 1e3 / args.steps
    t = torch.tensor([wall], dtype=torch.float64, device="cuda")
    if pg():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    value = npts * world * args.steps / wall
    # one PRG call per internal node of the tree: A, B (Hirose) or 4 AES-128 blocks (MMO)
    blocks = (4 if mmo else 2) * (npts - 1)
    peak = PEAK_MMO_BLOCKS if mmo else PEAK_TT_BLOCKS
    # a sample against the oracle (checker only): the first and last 4096 outputs
    out = {"metric": f"DCF full-domain evals/sec, N={nb} (not the BASELINE.json headline config)", "value": value,
           "unit": "evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "u8", "data": "synthetic",
           "config": {"workload": f"FD: full domain 2^{8 * nb} points, N={nb}, lambda={lam}, {prg_name}, 1 key, "
                                  f"party 0; replicas on {world} GPU(s)"},
           "roofline": {"bound": "lds", "engine": "ttable",
                        "kernel": ("k_fd_level16_mmo (8N launches)" if mmo
                                   else "k_prefix_build16 (levels 0..8N-5, one launch) + k_fd_dfs16<4, rows>"),
                        # HBM bytes: every output written once, plus (Hirose) the level-(8N-4) table rows
                        # written by the build and read back by the tail (32 B each)
                        "traffic": npts * lam + (0 if mmo else 2 * 32 * (npts >> 4)),
                        "traffic_source": "algorithmic bytes (no PMC profile of this launch shape)",
                        "achieved": blocks / kern_s / 1e9, "peak": peak / 1e9,
                        "measured_ceiling": None if mmo else measured_ceiling(blocks / kern_s),
                        "unit": f"G AES-{128 if mmo else 256} blocks/s", "frac": blocks / kern_s / peak, "kernel_ms": kern_s * 1e3,
                        "note": (f"{4 if mmo else 2} AES blocks per internal node (both children from one PRG "
                                 f"call), about {4 if mmo else 2} per leaf, vs {4 if mmo else 2} x 8N per point "
                                 "for pointwise eval")}}
    if rank == 0 and world == 1 and not args.no_cpu:  # cpu_baseline: rank 0 at N=1 only
        from oracle import oracle as O
        P = (O.OracleMmoPrg if mmo else O.OraclePrg)(keys, lam)
        cw = cwb.cpu().numpy().tobytes()
        k = O.OracleKey(nb, lam)
        n = 8 * nb
        k.cw_s[:] = np.frombuffer(cw[:n * lam], np.uint8).reshape(n, lam)
        k.cw_v[:] = np.frombuffer(cw[n * lam:2 * n * lam], np.uint8).reshape(n, lam)
        k.cw_t[:] = np.frombuffer(cw[2 * n * lam:2 * n * lam + n], np.uint8)
        off = dcf_amd.cwb_np1_offset(nb, lam, 1)
        k.cw_np1[:] = np.frombuffer(cw[off:off + lam], np.uint8)
        idx = np.concatenate([np.arange(4096), np.arange(npts - 4096, npts)])
        xs = np.array([list(int(i).to_bytes(nb, "big")) for i in idx], np.uint8)
        want = O.eval_(P, 0, k, seeds[0].cpu().numpy().tobytes(), xs, nthreads=8)
        got = ys[torch.from_numpy(idx).cuda()].cpu().numpy()
        out["matches_oracle_sample"] = bool(np.array_equal(got, want))
    return out


def run_latency(args, world, rank):
    """benches/dcf.rs: one gen, and one eval of ONE point, per call (criterion's bench_gen /
    bench_eval, N = 16, lambda = 16) through the host-pointer entry points a Rust caller's
    DcfHip would use (dcf_gen / dcf_eval: H2D, kernel, D2H, stream sync).  Reported as
    microseconds per call, with and without building the PRG inside the call as the
    reference's bench does (Aes256HirosePrg::new + DcfImpl::new per iteration; here that is
    dcf_prg_new: key schedules, tables and device buffers).  CPU beside it: the C restatement,
    1 thread, same calls.  Latency, not throughput: the GPU's launch and PCIe round trips
    bound it."""
    from oracle import oracle as O
    nb, lam = 16, 16
    rng = np.random.default_rng(0xDCF0005)
    keys = [rng.bytes(32) for _ in range(2)]
    dev = torch.cuda.current_device()
    prg = dcf_amd.Aes256HirosePrg(keys, lam, device=dev)
    d = dcf_amd.DcfImpl(nb, lam, prg)
    s0s = [rng.bytes(lam), rng.bytes(lam)]
    f = dcf_amd.CmpFn(rng.bytes(nb), rng.bytes(lam))
    k = d.gen(f, s0s, dcf_amd.BoundState.LtBeta)
    share0 = dcf_amd.Share([s0s[0]], k.cws, k.cw_np1)
    x = [rng.bytes(nb)]
    iters = max(50, args.steps * 40)

    def per_call(fn, n):
        for _ in range(max(5, n // 10)):
            fn()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        return (time.perf_counter() - t0) / n * 1e6

    # the C ABI calls a Rust DcfHip makes (dcf_gen / dcf_eval on host buffers), buffers packed once
    from dcf_amd._lib import check
    from dcf_amd.dcf import _ptr
    lib = dcf_amd.load()
    h = prg.handle
    a_b, b_b, s0_b, s1_b = bytes(f.alpha), bytes(f.beta), bytes(s0s[0]), bytes(s0s[1])
    cwb = np.frombuffer(dcf_amd.share_to_cwb(k, nb, lam), np.uint8).copy()
    cw_out = np.zeros_like(cwb)
    xb = np.frombuffer(x[0], np.uint8).copy()
    yb = np.zeros(lam, np.uint8)

    def c_gen():
        check(lib.dcf_gen(h, nb, _ptr(a_b), _ptr(b_b), _ptr(s0_b), _ptr(s1_b), 0, _ptr(cw_out)))

    def c_eval():
        check(lib.dcf_eval(h, nb, 0, _ptr(cwb), cwb.size, _ptr(s0_b), _ptr(xb), 1, _ptr(yb), lam))

    gen_us = per_call(c_gen, iters)
    eval_us = per_call(c_eval, iters)
    assert np.array_equal(cw_out, cwb), "dcf_gen bytes differ from DcfImpl.gen's"
    y_gpu = yb.reshape(1, lam).copy()
    py_gen_us = per_call(lambda: d.gen(f, s0s, dcf_amd.BoundState.LtBeta), max(20, iters // 4))
    py_eval_us = per_call(lambda: d.eval(False, share0, x), max(20, iters // 4))

    def gen_fresh():
        pr = dcf_amd.Aes256HirosePrg(keys, lam, device=dev)
        dcf_amd.DcfImpl(nb, lam, pr).gen(f, s0s, dcf_amd.BoundState.LtBeta)  # pr freed on return

    def eval_fresh():
        pr = dcf_amd.Aes256HirosePrg(keys, lam, device=dev)
        dcf_amd.DcfImpl(nb, lam, pr).eval(False, share0, x)  # pr freed on return

    gen_fresh_us = per_call(gen_fresh, max(20, iters // 20))
    eval_fresh_us = per_call(eval_fresh, max(20, iters // 20))
    P = O.OraclePrg(keys, lam)
    ok = O.gen(P, f.alpha, f.beta, s0s[0], s0s[1], 0)
    xs = np.frombuffer(x[0], np.uint8).reshape(1, nb).copy()
    cpu_gen_us = per_call(lambda: O.gen(P, f.alpha, f.beta, s0s[0], s0s[1], 0), iters)
    cpu_eval_us = per_call(lambda: O.eval_(P, 0, ok, s0s[0], xs, nthreads=1), iters)
    match = bool(np.array_equal(np.asarray(y_gpu), O.eval_(P, 0, ok, s0s[0], xs, nthreads=1)))
    return {"metric": "benches/dcf.rs latency: one gen / one single-point eval per call (us)", "value": eval_us,
            "unit": "us per single-point eval (host path)", "n_gpus": 1, "steps": iters, "warmup": iters // 10,
            "ms_per_step": eval_us / 1e3, "higher_is_better": False, "scaling": "none", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": "LAT: benches/dcf.rs bench_gen / bench_eval, N=16, lambda=16, Aes256HirosePrg "
                                   "(2 AES keys), one key, one point, host buffers", "n_bytes": nb, "lambda": lam},
            "gen_us": gen_us, "eval_us": eval_us, "python_api_gen_us": py_gen_us, "python_api_eval_us": py_eval_us,
            "gen_with_prg_new_us": gen_fresh_us, "eval_with_prg_new_us": eval_fresh_us,
            "cpu_baseline": {"gen_us": cpu_gen_us, "eval_us": cpu_eval_us, "cores": 1, "kind": "port",
                             "sample": f"{iters} calls each, the C restatement with AES-NI, 1 thread",
                             "matches_gpu": match},
            "note": "latency-bound: a tiny call is ONE launch of a latency kernel (kernels_lat.h: the AES of a "
                    "block on a 16-lane row; k_eval16_row2 — two levels per AES chain on right steps — / "
                    "k_gen16_row) that reads the key and points from, and writes its outputs to, a mapped pinned "
                    "buffer, plus one stream sync; a lone point's 8N levels run back to back (~0.5 us per level); "
                    "batch the points (C1) for throughput"}


def json_stdout():
    """The JSON line's stream.  File descriptor 1 is pointed at stderr for the rest of the run,
    so that nothing a library prints on stdout (RCCL's version banner at communicator init)
    can land beside the one JSON line the driver parses."""
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: this process starts the N ranks itself and exits with their status
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    out_stream = json_stdout()
    world, rank, _ = dist_setup(args.gpus, args.dist_backend, args.force_dist)
    if args.workload == "lat":
        out = run_latency(args, world, rank)
    elif args.workload == "c5":
        out = run_c5(args, world, rank)
    elif args.workload == "fd":
        out = run_fd(args, world, rank)
    else:
        out = run_eval(args, world, rank)
    if args.workload not in ("fd", "lat") and (args.workload != "c3" or args.prg != "hirose"):
        out["metric"] = (f"DCF evals/sec, workload {args.workload.upper()}, {args.prg} PRG "
                         "(not the BASELINE.json headline config)")
    if rank == 0:
        print(json.dumps(out), file=out_stream, flush=True)
    if pg():
        dist.barrier()
        dist.destroy_process_group()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=["c1", "c2", "c3", "c4", "c5", "fd", "lat"])
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--n-bytes", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--eval-mode", type=int, default=0, choices=[0, 1, 4],
                    help="LAMBDA = 16 AES engine: 0 auto, 1 lockstep T-table, 4 stream")
    ap.add_argument("--prg", default="hirose", choices=["hirose", "mmo"],
                    help="hirose: the reference's Aes256HirosePrg; mmo: Aes128MatyasMeyerOseasPrg (lambda = 16)")
    ap.add_argument("--prefix", type=int, default=-1,
                    help="shared-prefix table depth for single-key eval: -1 auto (library default), 0 off")
    ap.add_argument("--no-compare", action="store_true", help="skip the no-prefix comparison timing")
    ap.add_argument("--scaling", default=None, choices=["strong", "weak"],
                    help="strong: the workload's points (C5: keys) are split over the ranks (default for c3, c5); "
                         "weak: every rank gets the full count (default otherwise)")
    ap.add_argument("--host-path", action="store_true",
                    help="also time dcf_eval on host buffers (PCIe included; always on for c1)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo: CPU rehearsal)")
    ap.add_argument("--force-dist", action="store_true",
                    help="bring the process group up at N = 1 too (RCCL key broadcast, per-rank gather, "
                         "timing all-reduce run as at N > 1)")
    ap.add_argument("--check", action="store_true",
                    help="after timing, rank 0 re-evaluates every rank's slice and compares output digests")
    ap.add_argument("--abi-check", action="store_true",
                    help="run multi_gpu_abi_check at N = 1 too (always on at N > 1 for c1-c4)")
    args = ap.parse_args(argv)
    if args.scaling is None:
        args.scaling = "strong" if args.workload in ("c3", "c5") else "weak"
    args.lam = 16
    if args.workload == "c1":    # benches/dcf_batch_eval.rs:17 shape
        args.n_bytes = args.n_bytes or 16
        args.points = args.points or 100_000
    elif args.workload == "c2":  # 32-bit input
        args.n_bytes = args.n_bytes or 4
        args.points = args.points or (1 << 24)
    elif args.workload == "fd":  # full domain of a 32-bit input
        args.n_bytes = args.n_bytes or 4
    elif args.workload == "c4":  # benches/dcf_large_lambda.rs:10-11 shape, 2^22 points per GPU
        args.n_bytes = args.n_bytes or 16
        args.points = args.points or (1 << 22)
        args.lam = 16384
    else:
        args.n_bytes = args.n_bytes or 16
        args.points = args.points or (1 << 28)
    return args


if __name__ == "__main__":
    main()
