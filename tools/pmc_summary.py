"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv):
mean counter value per dispatch for each kernel, plus derived HBM bytes with the gfx950
FETCH_SIZE correction (MI355X_MICROARCH.md, HBM: FETCH_SIZE reports half the bytes of a wide
coalesced read; WRITE_SIZE is exact for 16-B stores).  FETCH_SIZE / WRITE_SIZE are in KB."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root):
    vals = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            meta[k] = dict(vgpr=int(row["VGPR_Count"]), agpr=int(row["Accum_VGPR_Count"]), sgpr=int(row["SGPR_Count"]),
                           lds=int(row["LDS_Block_Size"]), wg=int(row["Workgroup_Size"]), grid=int(row["Grid_Size"]))
    return vals, meta


def main(root="gpurun_out/pmc", match=None):
    vals, meta = load(root)
    out = {}
    for k, cs in vals.items():
        if match and match not in k:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dict(meta[k])
        d["counters"] = m
        if "FETCH_SIZE" in m:
            d["hbm_read_bytes_corrected"] = 2 * 1024 * m["FETCH_SIZE"]
        if "WRITE_SIZE" in m:
            d["hbm_write_bytes"] = 1024 * m["WRITE_SIZE"]
        if "TCC_HIT_sum" in m and m.get("TCC_MISS_sum") is not None:
            t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            d["l2_hit_rate"] = m["TCC_HIT_sum"] / t if t else None
        if "GRBM_GUI_ACTIVE" in m:
            d["gui_active_cycles_per_xcd"] = m["GRBM_GUI_ACTIVE"] / 8
        out[k] = d
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:])
