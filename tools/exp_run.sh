set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -30 $O/$n.log; exit $rc; }; }
B4="python bench.py --no-cpu-baseline --prefill-tokens 0"
B32="python bench.py --workload mistral-7b-f16-32k --steps 64 --no-cpu-baseline --prefill-tokens 0"
export XALM_HIP_LIB=xalm_amd/lib/var_sm.so
r test_sm python -u -m pytest tests/test_forward_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not persistent and not col"
for i in 1 2; do
  unset XALM_HIP_LIB; r b4_base_$i $B4; r b32_base_$i $B32
  export XALM_HIP_LIB=xalm_amd/lib/var_sm.so; r b4_sm_$i $B4; r b32_sm_$i $B32
done
