set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -30 $O/$n.log; exit $rc; }; }
r test_gq python -u -m pytest tests/test_gq_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
r bench_q8_0 python3 bench.py --workload mistral-7b-q8_0 --no-cpu-baseline
r bench_q4_0 python3 bench.py --workload mistral-7b-q4_0 --no-cpu-baseline
tail -1 $O/bench_q8_0.log > $O/bench_q8_0.json; tail -1 $O/bench_q4_0.log > $O/bench_q4_0.json
