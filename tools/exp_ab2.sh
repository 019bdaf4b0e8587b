set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in ${VARS:-base:xalm_amd/lib/var_base.so new:xalm_amd/lib/libxalm_hip.so}; do
  IFS=: read n lib <<< "$v"
  for w in ${WL:-mistral-7b-f16 mistral-7b-f8}; do
    XALM_HIP_LIB=$lib timeout -k 10 200 python bench.py --workload $w --steps 128 --no-cpu-baseline --prefill-tokens 0 --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$rep $n $w', d['value'], d['ms_per_step'])"
  done
done; done
