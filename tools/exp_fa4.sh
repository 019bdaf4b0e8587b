#!/bin/bash
# prompt attention variants: 2048-token and long-history prefill
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/fa4
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in def ${VARS:-}; do
    lib=""; [ "$v" != def ] && lib=xalm_amd/lib/var_$v.so
    timeout -k 10 300 env XALM_HIP_LIB=$lib python3 bench.py --workload mistral-7b-f16-32k --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048 > $OUT/pf32k_$v.log 2>&1 || { tail -3 $OUT/pf32k_$v.log; exit 1; }
    timeout -k 10 300 env XALM_HIP_LIB=$lib python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 3 --prefill-tokens 2048 > $OUT/pf_$v.log 2>&1 || { tail -3 $OUT/pf_$v.log; exit 1; }
    python3 -c "import json;a=json.loads(open('$OUT/pf32k_$v.log').read().strip().splitlines()[-1]);b=json.loads(open('$OUT/pf_$v.log').read().strip().splitlines()[-1]);print('$v', a['prefill']['tok_s_by_attention'], b['prefill']['tok_s'])"
done
