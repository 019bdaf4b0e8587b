set -u
O=gpurun_out/exp; mkdir -p $O
r() { local n=$1; shift; echo "== $n"; timeout -k 10 600 "$@" > $O/$n.log 2>&1; local rc=$?; tail -1 $O/$n.log | cut -c1-250; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -30 $O/$n.log; exit $rc; }; }
r smoke python -c "import __graft_entry__ as g; g.smoke()"
r tests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
r b4 python bench.py --no-cpu-baseline --prefill-tokens 0
r b8 python bench.py --workload mistral-7b-f8 --no-cpu-baseline --prefill-tokens 0
r b32 python bench.py --workload mistral-7b-f16-32k --steps 64 --no-cpu-baseline --prefill-tokens 0
