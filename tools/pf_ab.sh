#!/bin/bash
# Same-box A/B of prompt-pass variants: 2048-token prefill tok/s per library (LIBS), ROUNDS times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${LIBS:-base}; do
    XALM_HIP_LIB=xalm_amd/lib/var_$v.so timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline \
      --kernel-iters 5 ${ARGS:-} > gpurun_out/pfab.json 2> gpurun_out/pfab.err || { echo "FAILED $v"; tail -5 gpurun_out/pfab.err; exit 1; }
    python3 -c "
import json; d = json.load(open('gpurun_out/pfab.json')); p = d['prefill']
print('$v', p.get('tok_s'), p.get('ms'), (p.get('perplexity') or {}).get('tok_s'), p.get('tok_s_by_attention'), flush=True)"
  done
done
