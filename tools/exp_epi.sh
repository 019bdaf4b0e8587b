#!/bin/bash
# fused GEMM epilogues: tests, prefill benches (default vs separate epilogues via the option)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/epi
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
step tests 900 python3 -u -m pytest tests/test_forward_gpu.py tests/test_gq_gpu.py tests/test_regimes_gpu.py -x -q --timeout 300 --timeout-method thread -k "prefill or epilogue or glu or option or perplexity or prompt"
step pf 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048
step pf8 300 python3 bench.py --workload mistral-7b-f8 --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048
step pfq4 300 python3 bench.py --workload mistral-7b-q4_0 --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048
tail -2 $OUT/tests.log
python3 - <<'PY'
import json
for n in ("pf", "pf8", "pfq4"):
    d = json.loads(open(f"gpurun_out/epi/{n}.log").read().strip().splitlines()[-1])
    print(n, d["prefill"]["tok_s"], d["prefill"].get("matmul_tflops"), d["prefill"]["perplexity"]["tok_s"])
PY
