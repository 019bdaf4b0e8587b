#!/bin/bash
# GPU-box check: smoke, GPU parity tests, bench, rocprof kernel trace.
# Each GPU step has its own time limit; a crash / abort / timeout (rc not 0 or 1) ends the run.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
    local name=$1 limit=$2
    shift 2
    echo "== $name (limit ${limit}s) $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
STEPS=${STEPS:-smoke tests bench prof}
for s in $STEPS; do
    case $s in
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) run pytest_gpu 900 python -m pytest tests -m gpu -q --timeout 300 -rf ;;
        bench) run bench 600 python bench.py ;;
        bench_split) run bench_split 600 python bench.py --fuse-attn-wo 0 ;;
        bench_f8) run bench_f8 600 python bench.py --workload mistral-7b-f8 ;;
        bench_32k) run bench_32k 600 python bench.py --workload mistral-7b-f16-32k --steps 64 ;;
        bench_llama) run bench_llama 600 python bench.py --workload llama3-8b-f16 ;;
        gemvbench) run gemvbench 300 ./tools/gemv_bench 40 3 ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
                  python bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-iters 50 ;;
    esac
done
echo "== done"
