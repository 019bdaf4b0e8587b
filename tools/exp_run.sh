set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 900 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -40 $O/$n.log; exit $rc; }; }
r smoke python -c "import __graft_entry__ as g; g.smoke()"
r tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs
r bench python bench.py
