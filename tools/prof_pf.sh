#!/bin/bash
# rocprofv3 kernel stats of a 2048-token prompt pass (f16)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/profpf
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p" -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 5 --prefill-tokens 2048 > "$OUT/p.log" 2>&1 || { tail -5 "$OUT/p.log"; exit 1; }
cp "$OUT/p/run_kernel_stats.csv" "$OUT/kernel_stats_prefill.csv"
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/profpf/kernel_stats_prefill.csv")))[:12]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["TotalDurationNs"]) / 1e6, 2))
PY
