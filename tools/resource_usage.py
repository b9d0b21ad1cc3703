"""Per-kernel resource usage of librafthip (VGPR/AGPR/SGPR, spills, scratch, LDS, occupancy)
from the compiler's -Rpass-analysis=kernel-resource-usage remarks.
Usage: python tools/resource_usage.py [out.txt]   (compiles rh_abi.hip for gfx950, device only)"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "raft-teststuff_amd", "csrc", "rh_abi.hip")
KEYS = [("VGPR", "VGPRs"), ("AGPR", "AGPRs"), ("SGPR", "TotalSGPRs"), ("scratch_B", "ScratchSize [bytes/lane]"),
        ("occ_waves_per_SIMD", "Occupancy [waves/SIMD]"), ("VGPR_spill", "VGPRs Spill"),
        ("SGPR_spill", "SGPRs Spill"), ("static_LDS_B", "LDS Size [bytes/block]")]


def main():
    p = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only",
                        "-c", "-o", "/dev/null", SRC, "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, check=True)
    rows = []
    for blk in p.stderr.split("remark: Function Name: ")[1:]:
        name = blk.split()[0]
        vals = {}
        for short, key in KEYS:
            m = re.search(re.escape(key) + r": (\S+)", blk)
            vals[short] = m.group(1) if m else "?"
        rows.append((name, vals))
    lines = ["kernel " + " ".join(k for k, _ in KEYS)]
    for name, v in rows:
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        lines.append(dem + " " + " ".join(v[k] for k, _ in KEYS))
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write("# hipcc -O3 --offload-arch=gfx950 -Rpass-analysis=kernel-resource-usage (tools/resource_usage.py)\n")
            fh.write(out + "\n")


if __name__ == "__main__":
    main()
