"""Print mean-per-dispatch PMC values of the eval kernels (PMC_KERNELS: comma-separated name
filters, default k_eval) in gpurun_out/<tag>/*/ (round-2/3 lease scripts pmc_engines.sh / pmc_stall.sh, in git history)."""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*/"))):
    for db in glob.glob(os.path.join(d, "*.db")):
        c = sqlite3.connect(db)
        agg = defaultdict(lambda: defaultdict(list))
        for k, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
            if any(f in k for f in os.environ.get("PMC_KERNELS", "k_eval").split(",")):
                agg[k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]][cn].append(v)
        for k, cs in agg.items():
            print(os.path.basename(d.rstrip("/")), k, {cn: "%.4g" % (sum(v) / len(v)) for cn, v in sorted(cs.items())})
