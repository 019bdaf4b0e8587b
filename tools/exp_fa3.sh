#!/bin/bash
# prompt attention: tests + 2048-token / long-history prefill, default build and variants
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/fa3
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
step tests 600 python3 -u -m pytest tests/test_regimes_gpu.py tests/test_forward_gpu.py -x -q --timeout 300 --timeout-method thread -k "prompt_attention or prefill"
for v in "" ${VARS:-}; do
    lib=""; [ -n "$v" ] && lib=xalm_amd/lib/var_$v.so
    step pf2048_$v 300 env XALM_HIP_LIB=$lib python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048
    step pf32k_$v 400 env XALM_HIP_LIB=$lib python3 bench.py --workload mistral-7b-f16-32k --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/fa3/pf*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    p = d.get("prefill") or {}
    print(f, p.get("tok_s"), p.get("tok_s_by_attention"))
PY
