"""HBM bytes per dispatch of each kernel from rocprofv3 --pmc passes, over the LAST n dispatches
of each kernel only (e.g. a run whose first calls take another path): FETCH_SIZE doubled (the
gfx950 correction of MI355X_MICROARCH.md), WRITE_SIZE as is, both KB.
usage: python tools/pmc_last.py PMC_DIR N [MATCH]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root, n, match=""):
    n = int(n)
    rows = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                rows[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, cs in rows.items():
        if min(len(v) for v in cs.values()) < n:     # a kernel of the set-up, not of every call
            continue
        d = {}
        for c, v in cs.items():
            v = [x for _, x in sorted(v)][-n:]
            d[c] = sum(v) / len(v)
        o = {"dispatches_used": n}
        if "FETCH_SIZE" in d:
            o["hbm_read_bytes_corrected"] = 2 * 1024 * d["FETCH_SIZE"]
        if "WRITE_SIZE" in d:
            o["hbm_write_bytes"] = 1024 * d["WRITE_SIZE"]
        out[k] = o
    tot_r = sum(v.get("hbm_read_bytes_corrected", 0) for v in out.values())
    tot_w = sum(v.get("hbm_write_bytes", 0) for v in out.values())
    out["total_per_call_MB"] = {"read": tot_r / 1e6, "write": tot_w / 1e6, "sum": (tot_r + tot_w) / 1e6}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:])
