set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; grep -o '"prefill": {[^}]*' $O/$n.log | cut -c1-90; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -30 $O/$n.log; exit $rc; }; }
for m in 1 2 3; do
  r pf16_$m python bench.py --no-cpu-baseline --steps 8 --prefill-mode $m
  r pf8_$m python bench.py --workload mistral-7b-f8 --no-cpu-baseline --steps 8 --prefill-mode $m
done
r pf16_1b python bench.py --no-cpu-baseline --steps 8 --prefill-mode 1 --prefill-tokens 2048
r pf16_2b python bench.py --no-cpu-baseline --steps 8 --prefill-mode 2 --prefill-tokens 2048
