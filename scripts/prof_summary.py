"""Summarise rocprofv3 (rocpd sqlite) outputs of `bash scripts/gpu.sh TAG profile W`.

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


def main(d, suffix=""):
    print(f"# rocprofv3 summary: {d} {suffix}\n")
    for db in glob.glob(os.path.join(d, "trace" + suffix, "*.db")):
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
    for sub in sorted(glob.glob(os.path.join(d, "pmc_*" + suffix))):
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


def pmc_traffic(d, kernel_prefix="k_eval16<0>", suffix=""):
    """Per-launch HBM bytes of the dominant kernel: 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B).
    kernel_prefix may name several kernels joined by '+': their per-dispatch means add up
    (one 'launch' = one call of each)."""
    out = {}
    for name, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        for db in glob.glob(os.path.join(d, name + suffix, "*.db")):
            c = sqlite3.connect(db)
            rows = list(c.execute("select kernel_name, counter_name, value from counters_collection"))
            tot = 0.0
            for kp in kernel_prefix.split("+"):
                mult = 1.0
                if "*" in kp:  # "2*k_eval16_stream": two dispatches of that kernel per launch
                    m, kp = kp.split("*", 1)
                    mult = float(m)
                vals = [v for k, cn, v in rows if short(k).startswith(kp) and cn == counter]
                if vals:
                    tot += mult * sum(vals) / len(vals)
            if tot:
                out[counter] = tot * 1024
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        out["read_bytes_corrected"] = 2 * out["FETCH_SIZE"]
        out["traffic_bytes"] = 2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]
        out["traffic_bytes_x1"] = out["FETCH_SIZE"] + out["WRITE_SIZE"]
    return out


def record_traffic(path, entry):
    """Add (or replace) one launch shape's entry in profiles/pmc_traffic.json (a list)."""
    import json
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        t = []
    t = t if isinstance(t, list) else [t]
    key = lambda e: (e.get("kernel"), e.get("points_per_launch"), e.get("n_bytes"), e.get("lambda"),  # noqa: E731
                     e.get("prefix_levels", 0))
    t = [e for e in t if key(e) != key(entry)] + [entry]
    with open(path, "w") as f:
        json.dump(t, f, indent=1)


if __name__ == "__main__":
    # prof_summary.py <run dir> [--suffix _c2]
    # prof_summary.py <run dir> --traffic <json> <kernel prefix(es)> <workload> <points> <n_bytes> <lambda>
    #                 <prefix_levels> <algorithmic bytes> [--suffix _c2]
    args = sys.argv[1:]
    suffix = ""
    if "--suffix" in args:
        i = args.index("--suffix")
        suffix = args[i + 1]
        del args[i:i + 2]
    if "--traffic" in args:
        i = args.index("--traffic")
        out, prefix, wl, pts, nb, lam, pfx, alg = args[i + 1:i + 9]
        t = pmc_traffic(args[0], prefix, suffix)
        t.update({"source": args[0] + "/" + suffix, "kernel": prefix, "workload": wl, "points_per_launch": int(pts),
                  "n_bytes": int(nb), "lambda": int(lam), "prefix_levels": int(pfx), "algorithmic_bytes": float(alg),
                  "command": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- "
                             f"python bench.py --workload {wl.lower()} --steps 2 --warmup 1 --no-cpu --no-compare"})
        record_traffic(out, t)
        print(t)
    else:
        main(args[0], suffix)
