set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# usage: WL="workloads" ARGS_A=".." ARGS_B=".." LIB_A=path LIB_B=path bash tools/ab.sh  (alternating A/B)
WL=${WL:-mistral-7b-f16 mistral-7b-f8}
for w in $WL; do for v in A B A B; do
  if [ $v = A ]; then a=${ARGS_A:-}; lib=${LIB_A:-}; else a=${ARGS_B:-}; lib=${LIB_B:-}; fi
  XALM_HIP_LIB=$lib timeout -k 10 200 python bench.py --workload $w $a --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 > gpurun_out/ab.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));k=d['kernels'];print('$w [$v: $a ${lib##*/}]', d['value'], d['ms_per_step'], 'w13', k['gemv_w13']['avg_us'], 'qkv', k['gemv_qkv']['avg_us'])"
done; done
