#!/bin/bash
# HBM traffic of the decode kernels from PMC counters (MI355X_MICROARCH.md, HBM section):
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), each its own rocprofv3 run with
# --kernel-trace only; summarised per kernel by tools/pmc_summary.py (FETCH_SIZE x2 on gfx950).
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    echo "== pass $c $(date +%T)"
    timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -d "$OUT/$c" -o run --output-format csv -- \
        python bench.py --steps 16 --warmup 2 --no-cpu-baseline --kernel-iters 10 > "$OUT/$c.log" 2>&1
    rc=$?
    echo "== pass $c rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$OUT/$c.log"; exit $rc; }
done
python tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
