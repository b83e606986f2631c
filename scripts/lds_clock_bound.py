"""Counter-backed LDS bound of a workload's kernels at the clock the chip held.

  python scripts/lds_clock_bound.py profiles/r06/r06c_prof_c4.md C4 profiles/r05/r05ap_prof_c3.md C3 ... \\
      > profiles/lds_clock_bound.json

Reads one `scripts/gpu.sh TAG profile W` summary (prof_summary.py markdown: the kernel trace's mean
duration per kernel and the SQ pass's SQ_LDS_IDX_ACTIVE / GRBM_GUI_ACTIVE means per dispatch) and,
per kernel that touches the LDS:

  lds_cycles_per_cu = SQ_LDS_IDX_ACTIVE / 256 CUs       (every LDS-array cycle, conflicts included)
  clock_hz          = GRBM_GUI_ACTIVE / 8 XCDs / mean duration
  bound_ms          = lds_cycles_per_cu / clock_hz      (the LDS array 100 % busy at that clock)

The workload's bound is the sum over its kernels (they run back to back on one stream); kernels
without LDS work (the t-vector repack) count at their measured duration.  It answers "how close to
the LDS wall, at the clock the chip actually ran, are the kernels", beside the line's nominal
roofline (2.4 GHz), which the measured clocks (2.09 GHz head, 1.68 GHz tail in r06c) do not reach.
"""
import json
import re
import sys

CUS, XCDS = 256, 8


def parse(md):
    avg, pmc = {}, {}
    for line in open(md):
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if len(cells) == 5 and re.match(r"^\d+$", cells[1] or "") and re.match(r"^[\d.]+$", cells[3] or ""):
            avg[cells[0]] = float(cells[3])  # kernel | calls | total ms | avg ms | %
        elif len(cells) == 5 and cells[1] in ("SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE", "SQ_INSTS_LDS"):
            pmc.setdefault(cells[0], {})[cells[1]] = float(cells[3])
    return avg, pmc


def bound(md, workload, kernels=("k_eval", "k_wpfx", "k_tvec", "k_prefix", "k_cw", "k_mk", "k_gen16<")):
    avg, pmc = parse(md)
    rows, total_ms, meas_ms = [], 0.0, 0.0
    for k, ms in avg.items():
        # the key's gen runs once outside the timed step (C1-C4); C5's batched gen is part of its step
        if not k.startswith(kernels) or (k.startswith("k_gen") and workload != "C5"):
            continue
        c = pmc.get(k, {})
        meas_ms += ms
        if c.get("SQ_LDS_IDX_ACTIVE") and c.get("GRBM_GUI_ACTIVE"):
            cyc = c["SQ_LDS_IDX_ACTIVE"] / CUS
            clk = c["GRBM_GUI_ACTIVE"] / XCDS / (ms * 1e-3)
            b = cyc / clk * 1e3
            rows.append({"kernel": k, "mean_ms": ms, "lds_cycles_per_cu": cyc, "clock_ghz": clk / 1e9,
                         "lds_busy": cyc / (c["GRBM_GUI_ACTIVE"] / XCDS), "bound_ms": b,
                         "bound_ms_at_2p4ghz": cyc / 2.4e9 * 1e3})
            total_ms += b
        else:
            rows.append({"kernel": k, "mean_ms": ms, "bound_ms": ms, "note": "no LDS work: counted as measured"})
            total_ms += ms
    return {"workload": workload, "source": md, "bound_ms": total_ms, "kernels_ms": meas_ms,
            "frac_of_kernels": total_ms / meas_ms if meas_ms else None,
            "bound_ms_at_2p4ghz": sum(r.get("bound_ms_at_2p4ghz", r["bound_ms"]) for r in rows),
            "kernels": rows,
            "note": "sum over the eval's kernels of SQ_LDS_IDX_ACTIVE / 256 CUs / (GRBM_GUI_ACTIVE / 8 XCDs / "
                    "mean duration): the LDS array 100 % busy at the clock each kernel ran at "
                    "(scripts/lds_clock_bound.py)"}


if __name__ == "__main__":
    # pairs of (profile summary, workload): python scripts/lds_clock_bound.py A.md C4 B.md C3 ...
    a = sys.argv[1:]
    print(json.dumps([bound(a[i], a[i + 1]) for i in range(0, len(a), 2)], indent=1))
