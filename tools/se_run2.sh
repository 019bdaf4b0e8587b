#!/bin/bash
# Stream engine A/B on the GPU box: parity tests, then trace + bench with K-step rotation on/off.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stream_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/se_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/se_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 0; do
  XALM_SE_ROTATE=$r timeout -k 10 200 python -u tools/se_trace.py --tokens 8 > gpurun_out/se_trace_r$r.log 2>&1
  rc=$?
  echo "trace rotate=$r rc=$rc"; head -5 gpurun_out/se_trace_r$r.log; grep "input wait avg\|XhError" gpurun_out/se_trace_r$r.log | head -5
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
XALM_SE_ROTATE=1 timeout -k 10 300 python -u bench.py --engine 2 --steps 64 --warmup 4 --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 > gpurun_out/se_bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/se_bench.log | cut -c1-300
exit $rc
