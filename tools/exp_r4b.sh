#!/bin/bash
# long-split attention on MFMA + prompt attention softmax: tests, attn_bench, 32k / 4k benches
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4b
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
step tests 900 python3 -u -m pytest tests/test_ops_gpu.py tests/test_forward_gpu.py tests/test_regimes_gpu.py -x -q --timeout 300 --timeout-method thread -k "mha or multi_split or long_context or ring_buffer or 32k or prompt_attention or engines_agree"
step attn_bench 120 ./tools/attn_bench 32768 x x
step b32k 400 python3 bench.py --workload mistral-7b-f16-32k --steps 32 --warmup 4 --no-cpu-baseline --kernel-iters 10 --prefill-tokens 2048
step b4k 300 python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --kernel-iters 10 --prefill-tokens 2048
for v in ${VARS:-}; do
    step pf_$v 300 env XALM_HIP_LIB=xalm_amd/lib/var_$v.so python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048
    step pf32k_$v 400 env XALM_HIP_LIB=xalm_amd/lib/var_$v.so python3 bench.py --workload mistral-7b-f16-32k --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048
done
grep -E "merged|stream  t1024 D2" $OUT/attn_bench.log
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4b/b*.log") + glob.glob("gpurun_out/r4b/pf*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    p = d.get("prefill") or {}
    print(f, d["value"], d["kernels"].get("attention"), p.get("tok_s"), p.get("tok_s_by_attention"))
PY
