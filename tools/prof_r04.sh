#!/bin/bash
# rocprofv3 kernel stats of the decode step (f16, fp8) and of a 2048-token prompt pass.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/prof4
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 limit=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
}
step dec_f16 300 rocprofv3 --kernel-trace --stats -d "$OUT/dec_f16" -o run --output-format csv -- \
    python3 bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-iters 50 --prefill-tokens 0
step dec_f8 300 rocprofv3 --kernel-trace --stats -d "$OUT/dec_f8" -o run --output-format csv -- \
    python3 bench.py --workload mistral-7b-f8 --steps 64 --warmup 4 --no-cpu-baseline --kernel-iters 50 --prefill-tokens 0
step prefill_f16 300 rocprofv3 --kernel-trace --stats -d "$OUT/pf_f16" -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 5 --prefill-tokens 2048
for d in dec_f16 dec_f8 pf_f16; do cp "$OUT/$d/run_kernel_stats.csv" "$OUT/${d}_kernel_stats.csv"; done
echo "== done"
