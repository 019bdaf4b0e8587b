set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base:xalm_amd/lib/libxalm_hip.so:1024 t1024d100:xalm_amd/lib/var_t1024d100.so:1024 t512d0:xalm_amd/lib/var_t512d0.so:512 t512d100:xalm_amd/lib/var_t512d100.so:512 t512d200:xalm_amd/lib/var_t512d200.so:512; do
  IFS=: read n lib th <<< "$v"
  for w in mistral-7b-f16 mistral-7b-f8; do
    echo "=== $n $w"
    XALM_HIP_LIB=$lib timeout -k 10 200 python tools/aw_trace.py --workload $w --aw-threads $th 2>&1 | grep -v amdgpu.ids | grep -E "signalled|wo (passed|staged|end)|scores done" || exit 1
  done
done
for rep in 1 2; do for v in base:xalm_amd/lib/libxalm_hip.so t1024d100:xalm_amd/lib/var_t1024d100.so t512d0:xalm_amd/lib/var_t512d0.so t512d100:xalm_amd/lib/var_t512d100.so t512d200:xalm_amd/lib/var_t512d200.so; do
  IFS=: read n lib <<< "$v"
  for w in mistral-7b-f16 mistral-7b-f8; do
    XALM_HIP_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --prefill-tokens 0 --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$rep $n $w', d['value'], d['ms_per_step'])"
  done
done; done
