#!/bin/bash
# W2 matvec shape variants: correctness tests (default build), f16 decode and kernel times
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/w2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_forward_gpu.py tests/test_ops_gpu.py tests/test_regimes_gpu.py -x -q --timeout 300 --timeout-method thread -k "w2 or matmul or forward or long_row or graph or llama or mistral or decode" > $OUT/tests.log 2>&1 || { tail -15 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in def ${VARS:-} def; do
    lib=""; [ "$v" != def ] && lib=xalm_amd/lib/var_$v.so
    timeout -k 10 300 env XALM_HIP_LIB=$lib python3 bench.py --steps 128 --warmup 8 --cpu-tokens 16 --kernel-iters 40 --prefill-tokens 0 > $OUT/b_$v.log 2>&1 || { tail -3 $OUT/b_$v.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/b_$v.log').read().strip().splitlines()[-1]);p=d['cpu_baseline']['parity'];print('$v', d['value'], d['kernels']['gemv_w2'], p['gpu_vs_oracle64_max_abs'], p['oracle32_vs_oracle64_max_abs'], p['greedy_tokens_agree'])"
done
