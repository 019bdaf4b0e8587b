set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -30 $O/$n.log; exit $rc; }; }
B4="python bench.py --no-cpu-baseline --prefill-tokens 0"
B8="python bench.py --workload mistral-7b-f8 --no-cpu-baseline --prefill-tokens 0"
for qw in 4096 2048 1536 1024; do
  export XALM_QKV_WAVES=$qw
  r b4_$qw $B4
  r b8_$qw $B8
done
export XALM_QKV_WAVES=4096; r b4_4096b $B4
export XALM_QKV_WAVES=2048; r b4_2048b $B4
