#!/bin/bash
# LDS-only barriers around the split softmax: tests, attn_bench timeline, 32k / 4k / fp8 decode
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4d
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 limit=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 "$OUT/$name.log"; exit $rc; fi
}
step tests 900 python3 -u -m pytest tests/test_ops_gpu.py tests/test_forward_gpu.py tests/test_regimes_gpu.py -x -q --timeout 300 --timeout-method thread -k "mha or multi_split or long_context or ring_buffer or 32k or engines_agree or graph or fused or forward_matches"
step attn_bench 120 ./tools/attn_bench 32768 x x
for v in def ${VARS:-}; do
    lib=""; [ "$v" != def ] && lib=xalm_amd/lib/var_$v.so
    step b32k_$v 300 env XALM_HIP_LIB=$lib python3 bench.py --workload mistral-7b-f16-32k --steps 48 --warmup 4 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 0
    step b4k_$v 300 env XALM_HIP_LIB=$lib python3 bench.py --steps 128 --warmup 8 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 0
    step b8_$v 300 env XALM_HIP_LIB=$lib python3 bench.py --workload mistral-7b-f8 --steps 128 --warmup 8 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 0
done
tail -3 $OUT/tests.log
grep -E "merged|round   t1024|timeline|stream  t1024 D2" $OUT/attn_bench.log
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4d/b*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"])
PY
