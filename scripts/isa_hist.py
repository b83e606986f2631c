"""Instruction histogram of one kernel in a gfx950 device assembly file.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -S -o dcf.s dcf_amd/csrc/dcf_hip.hip
  python scripts/isa_hist.py dcf.s k_eval16_stream ILi2ELb1ELb0   [--blocks]

Prints the kernel's VGPR/SGPR/spill counts and, per basic block, the counts of
VALU / LDS / VMEM / SALU instructions, so the hot loop's mix can be read off.
"""
import re
import sys
from collections import Counter


def kernel_body(lines, pats):
    start = None
    for i, l in enumerate(lines):
        if ":" in l and not l.startswith((".", "\t", " ")) and all(p in l.split(":")[0] for p in pats):
            start = i
            break
    if start is None:
        raise SystemExit("kernel not found")
    end = start + 1
    while end < len(lines) and not lines[end].startswith("\t.section") and ".Lfunc_end" not in lines[end]:
        end += 1
    name = lines[start].split(":")[0]
    meta = {}
    for l in lines[end:end + 200]:
        m = re.match(r"\s*\.set\s+" + re.escape(name) + r"\.(\w+),\s*(\S+)", l)
        if m:
            meta[m.group(1)] = m.group(2)
    return name, lines[start + 1:end], meta


def classify(op):
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, pats = sys.argv[1], [a for a in sys.argv[2:] if not a.startswith("--")]
    lines = open(path).read().splitlines()
    name, body, meta = kernel_body(lines, pats)
    print(name)
    print({k: meta.get(k) for k in ("num_vgpr", "num_agpr", "numbered_sgpr", "private_seg_size")})
    blocks, cur = [], ("entry", Counter(), Counter())
    for l in body:
        s = l.strip()
        if re.match(r"^\.LBB\S+:", s) or re.match(r"^\.L\S+:", s):
            blocks.append(cur)
            cur = (s[:-1], Counter(), Counter())
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        cur[1][classify(op)] += 1
        cur[2][op] += 1
    blocks.append(cur)
    tot, ops = Counter(), Counter()
    for b, c, o in blocks:
        tot.update(c)
        ops.update(o)
    print("total", dict(tot))
    if "--blocks" in sys.argv:
        for b, c, o in blocks:
            if sum(c.values()) > 20:
                print(f"{b:24s} {dict(c)}")
                print("   ", ", ".join(f"{k}:{v}" for k, v in o.most_common(14)))
    hot = max(blocks, key=lambda x: x[1]["lds"])
    print("hottest (most LDS):", hot[0], dict(hot[1]))
    print("   ", ", ".join(f"{k}:{v}" for k, v in hot[2].most_common(30)))
    spills = sum(v for k, v in ops.items() if "readlane" in k or "writelane" in k)
    print("v_readlane/v_writelane:", spills)


if __name__ == "__main__":
    main()
