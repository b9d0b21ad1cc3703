"""Per-launch durations of the hot kernels from a rocprofv3 --kernel-trace CSV, grouped by kernel
and grid size, plus the C2 solve launches that overlap no other kernel (the bench's serial pass).
Usage: python tools/launch_durations.py run_kernel_trace.csv [label]"""
import csv
import statistics
import sys


def main(path, label):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "rh::" not in name:
                continue
            grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            rows.append((name.split("(")[0], grid, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print(f"# rocprofv3 --kernel-trace of {label}: per launch by grid size (threads)")
    groups = {}
    for n, g, s, e in rows:
        groups.setdefault((n, g), []).append((e - s) / 1e3)
    for (n, g), d in sorted(groups.items()):
        print(f"{n:60s} grid {g:8d} launches {len(d):4d}  mean {statistics.mean(d):8.1f} us  median "
              f"{statistics.median(d):8.1f}  min {min(d):8.1f}")
    ev = sorted(rows, key=lambda r: r[2])
    alone = []
    for i, (n, g, s, e) in enumerate(ev):
        if n != "void rh::k_solve_lds<2, 512, false, 1>" or g != 262144:
            continue
        if any(o[2] < e and o[3] > s for j, o in enumerate(ev) if j != i):
            continue
        alone.append((e - s) / 1e3)
    if alone:
        print(f"\n# C2 solve launches (grid 262144) that overlap no other kernel (the serial pass): {len(alone)} "
              f"launches, mean {statistics.mean(alone):.1f} us, median {statistics.median(alone):.1f} us, "
              f"min {min(alone):.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "python3 bench.py")
