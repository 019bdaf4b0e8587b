set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -40 $O/$n.log; exit $rc; }; }
r test_gq python -u -m pytest tests/test_gq_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
for i in 1 2; do
  unset XALM_HIP_LIB; r q4_new_$i python bench.py --workload mistral-7b-q4_0 --no-cpu-baseline --prefill-tokens 0
  export XALM_HIP_LIB=xalm_amd/lib/var_q4base.so; r q4_base_$i python bench.py --workload mistral-7b-q4_0 --no-cpu-baseline --prefill-tokens 0
done
