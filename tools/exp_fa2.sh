#!/bin/bash
# prompt attention v2 (shared K/V tiles): parity tests, 2048-token prefill, long-history prefill,
# and the attn_bench head-major floor
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/fa2
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 limit=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python3 -u -m pytest tests/test_regimes_gpu.py -x -v --timeout 300 --timeout-method thread -k "prompt_attention"
step pf2048 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --kernel-iters 5 --prefill-tokens 2048
step pf32k 400 python3 bench.py --workload mistral-7b-f16-32k --steps 8 --warmup 2 --no-cpu-baseline --kernel-iters 5 --prefill-tokens 2048
step attn_bench 120 ./tools/attn_bench 32768 x x
python3 - <<'PY'
import json
for n in ("pf2048", "pf32k"):
    d = json.loads(open(f"gpurun_out/fa2/{n}.log").read().strip().splitlines()[-1])
    print(n, d["value"], json.dumps(d.get("prefill"))[:600])
PY
