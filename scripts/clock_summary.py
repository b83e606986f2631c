"""Per-kernel effective clock from GRBM_GUI_ACTIVE PMC runs (round-3 lease script pmc_clock.sh, in git history) (rocpd sqlite): mean
GRBM_GUI_ACTIVE per dispatch / 8 XCDs / mean kernel duration of the same run.

  python scripts/clock_summary.py gpurun_out/<tag>
"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

from prof_summary import short

XCDS = 8


def main(d):
    print(f"# effective engine clock per kernel: {d}\n")
    print("| run | kernel | dispatches | mean ms | mean GRBM_GUI_ACTIVE | GHz (/ 8 XCDs) |")
    print("|---|---|---|---|---|---|")
    for sub in sorted(glob.glob(os.path.join(d, "clk_*"))):
        if not os.path.isdir(sub):
            continue
        for db in glob.glob(os.path.join(sub, "**", "*.db"), recursive=True):
            c = sqlite3.connect(db)
            dur = defaultdict(list)
            for name, du in c.execute("select name, duration from kernels"):
                dur[short(name)].append(du)
            cyc = defaultdict(list)
            for kname, cname, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
                if cname == "GRBM_GUI_ACTIVE":
                    cyc[short(kname)].append(val)
            for k, vals in cyc.items():
                if k.startswith("__amd") or k not in dur:
                    continue
                ms = sum(dur[k]) / len(dur[k]) / 1e6  # kernels.duration is in ns
                g = sum(vals) / len(vals)
                ghz = g / XCDS / (ms * 1e-3) / 1e9 if ms > 0 else float("nan")
                print(f"| {os.path.basename(sub)} | {k} | {len(vals)} | {ms:.3f} | {g:.4g} | {ghz:.3f} |")


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(__file__))
    main(sys.argv[1])
