#!/bin/bash
# Stream engine on the GPU box: parity tests, trace, short bench (each step time-limited).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stream_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/se_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/se_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/se_trace.py --tokens 8 > gpurun_out/se_trace.log 2>&1
rc=$?
echo "trace rc=$rc"; cat gpurun_out/se_trace.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --engine 2 --steps 64 --warmup 4 --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 > gpurun_out/se_bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/se_bench.log | cut -c1-400
exit $rc
