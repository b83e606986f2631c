"""Same-lease C3 evidence: the driver's bench command and a rocprofv3 kernel trace of the same
workload taken in one gpurun call (`bash scripts/gpu.sh TAG trace`), reduced to one summary:

  python scripts/lease_c3.py gpurun_out/<tag> > profiles/<tag>_prof_c3.md

frac_profiled = AES blocks executed per eval call (the bench line's executed_blocks_per_eval x
2^28 points, table build included) / (mean k_eval16_stream + mean k_prefix_build16 duration
from the trace) / the 87.8 G blocks/s LDS peak, beside the bench line's frac (HIP events
around the whole call).  Both must fit under the line's ms_per_step.
"""
import glob
import json
import os
import sqlite3
import sys

from prof_summary import short

PEAK = 256 * 32 * 2.4e9 / 224


def main(d):
    line = json.loads(open(os.path.join(d, "bench_c3.json")).read().strip().splitlines()[-1])
    r = line["roofline"]
    m = line["config"]["points_per_gpu"]
    blocks = m * r["executed_blocks_per_eval"]
    db = glob.glob(os.path.join(d, "trace", "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average from top_kernels"))
    avg = {short(n): a / 1e3 for n, _, _, a in rows}  # top_kernels: microseconds -> ms
    walk = [v for k, v in avg.items() if k.startswith("k_eval16_stream")]
    table = [v for k, v in avg.items() if k.startswith("k_prefix_build16")]
    prof_ms = (walk[0] if walk else 0.0) + (table[0] if table else 0.0)
    frac_prof = blocks / (prof_ms * 1e-3) / PEAK if prof_ms else None
    print(f"# C3 same-lease evidence: {d}\n")
    print("Bench line (the driver's command, `python bench.py --gpus 1 --steps 20 --warmup 5`):\n")
    print(f"* value {line['value']:.4e} evals/s, ms_per_step {line['ms_per_step']:.2f}, kernel_ms (HIP events over "
          f"the eval call) {r['kernel_ms']:.2f}, frac {r['frac']:.4f}, executed blocks/eval "
          f"{r['executed_blocks_per_eval']:.3f}, prefix levels {r['prefix_levels']}")
    print("\nrocprofv3 --kernel-trace --stats of the same workload in the same lease "
          "(`bench.py --steps 5 --warmup 2 --no-cpu --no-compare`):\n")
    print("| kernel | calls | total ms | avg ms |")
    print("|---|---|---|---|")
    for n, calls, tot, a in rows:
        print(f"| {short(n)} | {calls} | {tot / 1e3:.3f} | {a / 1e3:.3f} |")
    print(f"\n* walk {walk[0] if walk else float('nan'):.3f} ms + table build "
          f"{table[0] if table else float('nan'):.3f} ms = {prof_ms:.3f} ms per eval call under the profiler "
          f"(<= ms_per_step {line['ms_per_step']:.3f}: {prof_ms <= line['ms_per_step']})")
    print(f"* frac_profiled = {blocks:.4e} blocks / {prof_ms:.3f} ms / {PEAK / 1e9:.2f} G blocks/s = "
          f"**{frac_prof:.4f}** (bench line frac {r['frac']:.4f})")
    json.dump({"frac": r["frac"], "frac_profiled": frac_prof, "profiled_ms": prof_ms, "ms_per_step": line["ms_per_step"],
               "kernel_ms": r["kernel_ms"], "value": line["value"]},
              open(os.path.join(d, "lease_c3.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
