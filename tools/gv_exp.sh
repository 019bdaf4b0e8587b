#!/bin/bash
# A/B of gemv launch variants (XALM_GV<epi>) in the real decode step; then the GPU parity
# tests with the variants on
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --prefill-tokens 0 --steps 256 --warmup 8 ${WL:-}"
run() { local name=$1; shift; echo "== $name $*"; env "$@" timeout -k 10 120 $B > gpurun_out/gv.tmp 2>&1 || { tail -5 gpurun_out/gv.tmp; exit 1; }; python3 -c "
import json
l=[x for x in open('gpurun_out/gv.tmp') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'])"; }
for spec in ${SPECS:-"base XALM_GV0=0"}; do
    IFS=, read -ra kv <<< "$spec"
    run "${kv[@]}"
done
if [ -n "${TESTENV:-}" ]; then
    echo "== tests with $TESTENV"
    env $TESTENV timeout -k 10 600 python -m pytest tests/test_forward_gpu.py tests/test_ops_gpu.py -m gpu -q -x --timeout 120 > gpurun_out/gv_tests.log 2>&1; rc=$?
    tail -3 gpurun_out/gv_tests.log; exit $rc
fi
