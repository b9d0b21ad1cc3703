"""HBM MB per launch of each rh:: kernel from tools/gpu.sh pmc passes
(gpurun_out/<dir>/pmc_<lib>_<workload>/{WRITE_SIZE,FETCH_SIZE}); FETCH_SIZE doubled per the
gfx950 correction (tools/pmc_summary.py)."""
import csv
import glob
import os
import sys
from collections import defaultdict

for d in sorted(glob.glob(os.path.join(sys.argv[1], "pmc_*"))):
    for g in ("WRITE_SIZE", "FETCH_SIZE"):
        f = os.path.join(d, g, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        v = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "rh::" in r["Kernel_Name"]:
                v[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
        k = 2 if g == "FETCH_SIZE" else 1
        print(os.path.basename(d), g, {n: round(k * 1024 * sum(x) / len(x) / 1e6, 1) for n, x in v.items()})
