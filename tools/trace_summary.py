"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, grouped by kernel name and grid.

    python tools/trace_summary.py gpurun_out/<dir>/run_kernel_trace.csv [name-substring] [top]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    agg = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if sub not in name:
                continue
            grid = r.get("Grid_Size_X", r.get("Grid_Size", ""))
            agg[f"{name.split('(')[0][:70]} grid{grid}"].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    total = 0.0
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        total += sum(v)
        print(f"{k:90s} n={len(v):6d} avg={sum(v) / len(v):9.2f}us sum={sum(v) / 1000:9.3f}ms")
    print(f"total (listed) {total / 1000:.3f} ms")


if __name__ == "__main__":
    main()
