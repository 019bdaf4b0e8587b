# A/B of gguf-block decode variants (alternating, one box): VARS="name:lib ..." WL="workloads"
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for v in ${VARS}; do
  IFS=: read n lib <<< "$v"
  for w in ${WL}; do
    XALM_HIP_LIB=$lib timeout -k 10 200 python bench.py --workload $w --steps 128 --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));k=d['kernels'];print('$rep $n $w', d['value'], d['ms_per_step'], 'w13', k['gemv_w13']['avg_us'], k['gemv_w13']['GBps'], 'w2', k['gemv_w2']['avg_us'])"
  done
done; done
