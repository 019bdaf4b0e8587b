set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in sf sfst5; do echo "== trace $v"; XLANDED=1 XALM_HIP_LIB=xalm_amd/lib/var_$v.so timeout -k 10 200 python tools/layer_trace.py --workload mistral-7b-f16 2>&1 | grep -v amdgpu.ids | grep -v boundary || exit 1; done
for rep in 1 2; do for v in base:xalm_amd/lib/libxalm_hip.so sf:xalm_amd/lib/var_sf.so sfxb:xalm_amd/lib/var_sfxb.so; do
  IFS=: read n lib <<< "$v"
  for w in mistral-7b-f16 mistral-7b-f8; do
    XALM_HIP_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --prefill-tokens 0 --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$rep $n $w', d['value'], d['ms_per_step'])"
  done
done; done
