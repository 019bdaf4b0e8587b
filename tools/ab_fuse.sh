set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# usage: WL="workloads" ARGS_A="..." ARGS_B="..." bash tools/ab_fuse.sh   (alternating A/B pairs)
WL=${WL:-mistral-7b-f16 mistral-7b-f8}
for w in $WL; do for v in A B A B; do
  if [ $v = A ]; then a=${ARGS_A:-}; else a=${ARGS_B:-}; fi
  timeout -k 10 200 python bench.py --workload $w $a --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 > gpurun_out/ab.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$w [$v: $a]', d['value'], d['ms_per_step'])"
done; done
