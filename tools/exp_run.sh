set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -30 $O/$n.log; exit $rc; }; }
B8="python bench.py --workload mistral-7b-f8 --no-cpu-baseline --prefill-tokens 0"
for i in 1 2 3; do
  unset XALM_HIP_LIB; r p7_$i $B8
  export XALM_HIP_LIB=xalm_amd/lib/var_np7.so; r np7_$i $B8
done
