set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for v in ${VARS}; do
  IFS=: read n lib <<< "$v"
  for w in ${WL:-mistral-7b-f8}; do
    XALM_HIP_LIB=$lib timeout -k 10 200 python bench.py --workload $w --steps 128 --no-cpu-baseline --prefill-tokens 0 --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$rep $n $w', d['value'], d['ms_per_step'])"
  done
done; done
