set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -40 $O/$n.log; exit $rc; }; }
r test_mha python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k mha
r tests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
r smoke python -c "import __graft_entry__ as g; g.smoke()"
r b32 python bench.py --workload mistral-7b-f16-32k --steps 64 --no-cpu-baseline --prefill-tokens 0
