#!/bin/bash
# Stream-engine experiments (XALM_SE_DEBUG bits, results invalid): time per token under each.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 8 10 11 15 14; do
  XALM_SE_DEBUG=$d timeout -k 10 120 python -u tools/se_trace.py --tokens 8 > gpurun_out/se_exp_$d.log 2>&1
  rc=$?
  echo "debug=$d rc=$rc $(head -1 gpurun_out/se_exp_$d.log)"
  grep "loader\|wave0\|input wait avg" gpurun_out/se_exp_$d.log | head -9
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
