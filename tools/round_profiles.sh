#!/bin/bash
# Round evidence on the GPU box: PMC traffic passes, rocprofv3 kernel stats, and bench lines for
# every BASELINE workload.  Output: gpurun_out/$ROUND/ (copy into profiles/ as ${ROUND}_*).
# Each GPU step has its own limit; a crash / abort / timeout ends the run.
set -u
cd "$(dirname "$0")/.."
ROUND=${ROUND:-r06}
PART=${PART:-all}   # a: tests, PMC, kernel trace, fp16 / fp8 benches; b: the other workloads
OUT=gpurun_out/$ROUND
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
if [ "$PART" != b ]; then
if [ -z "${SKIP_TESTS:-}" ]; then
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs
fi
# HBM traffic (MI355X_MICROARCH.md HBM section): FETCH_SIZE and WRITE_SIZE in separate passes
for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_$c 300 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc/$c" -o run --output-format csv -- \
        python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --kernel-iters 10 --prefill-tokens 0
    step pmc_f8_$c 300 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_f8/$c" -o run --output-format csv -- \
        python3 bench.py --workload mistral-7b-f8 --steps 16 --warmup 2 --no-cpu-baseline --kernel-iters 10 --prefill-tokens 0
done
python3 tools/pmc_summary.py "$OUT/pmc" "$OUT/pmc_f8" > "$OUT/pmc.json"
cp "$OUT/pmc.json" "profiles/${ROUND}_pmc.json"   # read by bench.py's roofline.traffic
step kernel_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-iters 50 --prefill-tokens 0
cp "$OUT/prof/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
step kernel_trace_f8 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_f8" -o run --output-format csv -- \
    python3 bench.py --workload mistral-7b-f8 --steps 64 --warmup 4 --no-cpu-baseline --kernel-iters 50 --prefill-tokens 0
cp "$OUT/prof_f8/run_kernel_stats.csv" "$OUT/kernel_stats_f8.csv"
step kernel_trace_prefill 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_pf" -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 5 --prefill-tokens 2048
cp "$OUT/prof_pf/run_kernel_stats.csv" "$OUT/kernel_stats_prefill.csv"
step bench 600 python3 bench.py
step bench_f8 600 python3 bench.py --workload mistral-7b-f8
# configs[1]'s worst tokens: a synthetic history up to pos 3800, the timed tokens end at kv_len 4096
step bench_kv4k 300 python3 bench.py --pos0 3800 --prefill-tokens 0
step kernel_trace_kv4k 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_kv4k" -o run --output-format csv -- \
    python3 bench.py --pos0 3800 --steps 256 --warmup 8 --no-cpu-baseline --kernel-iters 20 --prefill-tokens 0
cp "$OUT/prof_kv4k/run_kernel_stats.csv" "$OUT/kernel_stats_kv4k.csv"
fi
if [ "$PART" != a ]; then
step kernel_trace_32k 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_32k" -o run --output-format csv -- \
    python3 bench.py --workload mistral-7b-f16-32k --steps 32 --warmup 4 --no-cpu-baseline --kernel-iters 20 --prefill-tokens 0
cp "$OUT/prof_32k/run_kernel_stats.csv" "$OUT/kernel_stats_32k.csv"
step kernel_trace_llama 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_llama" -o run --output-format csv -- \
    python3 bench.py --workload llama3-8b-f16 --steps 64 --warmup 4 --no-cpu-baseline --kernel-iters 50 --prefill-tokens 0
cp "$OUT/prof_llama/run_kernel_stats.csv" "$OUT/kernel_stats_llama.csv"
step kernel_trace_q4_0 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_q4" -o run --output-format csv -- \
    python3 bench.py --workload mistral-7b-q4_0 --steps 64 --warmup 4 --no-cpu-baseline --kernel-iters 50 --prefill-tokens 0
cp "$OUT/prof_q4/run_kernel_stats.csv" "$OUT/kernel_stats_q4_0.csv"
step bench_32k 900 python3 bench.py --workload mistral-7b-f16-32k --steps 64 --cpu-tokens 8
step bench_llama 600 python3 bench.py --workload llama3-8b-f16
# SURVEY 8f-4 block formats (not BASELINE configs): a shorter CPU sample (the fp64 parity
# evaluation decodes every block element scalar, as quants.py dequantizes it)
step bench_q8_0 600 python3 bench.py --workload mistral-7b-q8_0 --cpu-tokens 64
step bench_q4_0 600 python3 bench.py --workload mistral-7b-q4_0 --cpu-tokens 64
fi
for b in bench bench_f8 bench_kv4k bench_32k bench_llama bench_q8_0 bench_q4_0; do [ -f "$OUT/$b.log" ] && tail -1 "$OUT/$b.log" > "$OUT/$b.json"; done
echo "== done"
