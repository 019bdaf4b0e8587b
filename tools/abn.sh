#!/bin/bash
# Interleaved same-box A/B/... of library variants (tools/build_variant.sh NAME -> xalm_amd/lib/var_NAME.so):
#   LIBS="base xbar" WL="mistral-7b-f16 mistral-7b-f8" ROUNDS=2 bash tools/abn.sh
# One decode bench per (round, workload, variant); prints tok/s and the per-launch kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=${LIBS:-base}
WL=${WL:-mistral-7b-f16}
ROUNDS=${ROUNDS:-2}
STEPS=${STEPS:-256}
for r in $(seq 1 "$ROUNDS"); do
  for w in $WL; do
    for v in $LIBS; do
      XALM_HIP_LIB=xalm_amd/lib/var_$v.so timeout -k 10 200 python3 bench.py --workload "$w" --steps "$STEPS" \
        --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 ${ARGS:-} > gpurun_out/abn.json 2> gpurun_out/abn.err || {
        echo "FAILED $w $v rc=$?"; tail -5 gpurun_out/abn.err; exit 1; }
      python3 - "$w" "$v" <<'EOF'
import json, sys
d = json.load(open('gpurun_out/abn.json'))
k = d['kernels']
print(f"{sys.argv[1]:18s} {sys.argv[2]:10s} {d['value']:8.2f} tok/s {d['ms_per_step']:.4f} ms  " +
      " ".join(f"{n[5:] if n.startswith('gemv_') else n} {v['avg_us']:.2f}" for n, v in k.items()), flush=True)
EOF
    done
  done
done
