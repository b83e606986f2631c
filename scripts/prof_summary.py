"""Summarise rocprofv3 (rocpd sqlite) outputs of scripts/gpu_profile.sh.

  python scripts/prof_summary.py gpurun_out/r01 > profiles/r01_summary.md

Kernel stats come from --kernel-trace --stats (top_kernels / kernels views);
PMC values from the separate --pmc passes (counters_collection view), per
dispatch of each kernel.  HBM bytes follow MI355X_MICROARCH.md §HBM:
FETCH_SIZE (KiB) reports half the bytes of wide streaming reads on gfx950, so
the corrected read figure is 2 x FETCH_SIZE; WRITE_SIZE is taken as is.
"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:80]


def main(d):
    print(f"# rocprofv3 summary: {d}\n")
    for db in glob.glob(os.path.join(d, "trace", "*.db")):
        c = sqlite3.connect(db)
        print("## kernel trace (--kernel-trace --stats)\n")
        print("| kernel | calls | total ms | avg ms | % |")
        print("|---|---|---|---|---|")
        for name, calls, tot, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            # top_kernels durations are in microseconds
            print(f"| {short(name)} | {calls} | {tot / 1e3:.3f} | {avg / 1e3:.3f} | {pct:.2f} |")
        print()
        rows = list(c.execute("select name, duration, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, "
                              "grid_x, workgroup_x from kernels"))
        seen = set()
        print("| kernel | grid | wg | VGPR | AGPR | SGPR | LDS B |")
        print("|---|---|---|---|---|---|---|")
        for name, dur, v, a, s, lds, gx, wx in rows:
            k = short(name)
            if k in seen:
                continue
            seen.add(k)
            print(f"| {k} | {gx} | {wx} | {v} | {a} | {s} | {lds} |")
        print()
    for sub in sorted(glob.glob(os.path.join(d, "pmc_*"))):
        for db in glob.glob(os.path.join(sub, "*.db")):
            c = sqlite3.connect(db)
            agg = defaultdict(lambda: defaultdict(list))
            for kname, cname, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
                agg[short(kname)][cname].append(val)
            print(f"## PMC pass {os.path.basename(sub)} (mean per dispatch)\n")
            print("| kernel | counter | dispatches | mean | derived |")
            print("|---|---|---|---|---|")
            for k, cs in agg.items():
                if k.startswith("__amd") or "distribution" in k:
                    continue
                for cname, vals in cs.items():
                    mean = sum(vals) / len(vals)
                    extra = ""
                    if cname == "FETCH_SIZE":
                        extra = f"corrected read bytes = 2 x {mean:.0f} KiB = {2 * mean * 1024 / 1e9:.3f} GB"
                    elif cname == "WRITE_SIZE":
                        extra = f"{mean * 1024 / 1e9:.3f} GB"
                    print(f"| {k} | {cname} | {len(vals)} | {mean:.4g} | {extra} |")
            print()


def pmc_traffic(d, kernel_prefix="k_eval16<0>"):
    """Per-launch HBM bytes of the dominant kernel: 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B)."""
    out = {}
    for name, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        for db in glob.glob(os.path.join(d, name, "*.db")):
            c = sqlite3.connect(db)
            vals = [v for k, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection")
                    if short(k).startswith(kernel_prefix) and cn == counter]
            if vals:
                out[counter] = sum(vals) / len(vals) * 1024
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        out["read_bytes_corrected"] = 2 * out["FETCH_SIZE"]
        out["traffic_bytes"] = 2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]
    return out


if __name__ == "__main__":
    # prof_summary.py <run dir> [<pmc_traffic.json out> <kernel prefix>]
    main(sys.argv[1])
    if len(sys.argv) > 2:
        import json
        prefix = sys.argv[3] if len(sys.argv) > 3 else "k_eval16_stream"
        t = pmc_traffic(sys.argv[1], prefix)
        t["source"] = sys.argv[1]
        t["kernel"] = prefix
        # the launch shape of scripts/gpu_profile.sh's bench run (bench.py defaults, workload C3)
        # auto shared-prefix depth 26: x (16 B) + y (16 B) + one 32-byte table row per point
        t.update({"workload": "C3", "points_per_launch": 1 << 28, "n_bytes": 16, "lambda": 16,
                  "prefix_levels": 26, "algorithmic_bytes": (1 << 28) * 64,
                  "command": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- "
                             "python bench.py --steps 2 --warmup 1 --no-cpu"})
        with open(sys.argv[2], "w") as f:
            json.dump(t, f, indent=1)
