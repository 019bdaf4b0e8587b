set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -30 $O/$n.log; exit $rc; }; }
B4="python bench.py --no-cpu-baseline --prefill-tokens 0"
B8="python bench.py --workload mistral-7b-f8 --no-cpu-baseline --prefill-tokens 0"
for v in p1 p2; do
  export XALM_HIP_LIB=xalm_amd/lib/var_$v.so
  for mb in 0 16 32 48; do
    export XALM_AW_PF_MB=$mb
    r b4_${v}_$mb $B4
    python -c "import json;d=json.load(open('$O/b4_${v}_$mb.log'.replace('.log','.log'))) if False else None" 2>/dev/null
    grep -o '"gemv_w13": {[^}]*}' $O/b4_${v}_$mb.log
  done
  export XALM_AW_PF_MB=16; r b8_${v}_16 $B8
  export XALM_AW_PF_MB=0; r b8_${v}_0 $B8
done
