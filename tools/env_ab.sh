#!/bin/bash
# Alternating A/B of runtime environment settings on the decode bench (no code change).
# usage: ENV_B="HIP_FORCE_DEV_KERNARG=1" WL="mistral-7b-f16" bash tools/env_ab.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
WL=${WL:-mistral-7b-f16}
for w in $WL; do for v in A B A B; do
  if [ $v = A ]; then e=${ENV_A:-XALM_NOP=1}; else e=${ENV_B:-XALM_NOP=1}; fi
  env $e timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 > gpurun_out/envab.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/envab.json'));k=d['kernels'];print('$w [$v: $e]', d['value'], d['ms_per_step'], 'w13', k['gemv_w13']['avg_us'], 'qkv', k['gemv_qkv']['avg_us'])"
done; done
