"""Per-kernel registers / spills from `hipcc -Rpass-analysis=kernel-resource-usage` output.
  python scripts/ru_summary.py remarks.txt [substring ...]"""
import re
import sys

txt = open(sys.argv[1]).read()
keys = sys.argv[2:]
for b in re.split(r"remark: [^\n]*Function Name: ", txt)[1:]:
    name = b.split("\n")[0].strip()
    if keys and not any(k in name for k in keys):
        continue

    def g(k):
        m = re.search(re.escape(k) + r": (\S+)", b)
        return m.group(1) if m else "?"
    print("%-100s V%s S%s scratch%s vspill%s sspill%s" % (name[:100], g("VGPRs"), g("SGPRs"),
          g("ScratchSize [bytes/lane]"), g("VGPRs Spill"), g("SGPRs Spill")))
