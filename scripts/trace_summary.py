"""Kernel-trace summary of a rocprofv3 run (ROCm 7.2 writes its results as a SQLite database,
`<dir>/<...>_results.db`): calls / total / average / min / max per kernel, and the per-dispatch
timeline of the last `--tail` dispatches.

  python scripts/trace_summary.py gpurun_out/r04b/trace_c4 [--tail 12] > profiles/r04b_prof_c4.md
"""
import argparse
import collections
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path", help="rocprofv3 output directory (or the .db file)")
    ap.add_argument("--tail", type=int, default=12)
    a = ap.parse_args()
    dbs = [a.path] if a.path.endswith(".db") else sorted(glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True))
    if not dbs:
        raise SystemExit(f"no .db under {a.path}")
    rows = []
    for db in dbs:
        c = sqlite3.connect(db)
        rows += list(c.execute("select name, start, end, grid_x, workgroup_x, vgpr_count, sgpr_count, lds_size "
                               "from kernels order by start"))
    d = collections.defaultdict(list)
    meta = {}
    for n, s, e, gx, wx, vg, sg, lds in rows:
        d[n].append((e - s) / 1e6)
        meta[n] = (gx, wx, vg, sg, lds)
    print(f"# rocprofv3 kernel trace: {a.path}\n")
    print("| kernel | calls | total ms | avg ms | min ms | max ms | % |")
    print("|---|---|---|---|---|---|---|")
    tot = sum(sum(v) for v in d.values())
    for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"| {n[:90]} | {len(v)} | {sum(v):.3f} | {sum(v) / len(v):.3f} | {min(v):.3f} | {max(v):.3f} | "
              f"{100 * sum(v) / tot:.2f} |")
    print("\n| kernel | grid | wg | VGPR | SGPR | LDS B |\n|---|---|---|---|---|---|")
    for n, (gx, wx, vg, sg, lds) in meta.items():
        print(f"| {n[:90]} | {gx} | {wx} | {vg} | {sg} | {lds} |")
    print(f"\n## last {a.tail} dispatches (ms from the first of them)\n")
    print("| kernel | start ms | duration ms |\n|---|---|---|")
    last = rows[-a.tail:]
    t0 = last[0][1] if last else 0
    for n, s, e, *_ in last:
        print(f"| {n[:90]} | {(s - t0) / 1e6:.3f} | {(e - s) / 1e6:.3f} |")


if __name__ == "__main__":
    main()
