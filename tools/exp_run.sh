set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -40 $O/$n.log; exit $rc; }; }
r test_gq python -u -m pytest tests/test_gq_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
