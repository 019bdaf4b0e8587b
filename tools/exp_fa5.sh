#!/bin/bash
# prompt attention: 2 tiles per ring stage vs 1 — parity tests, then long-history / 2048 prefill
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_regimes_gpu.py tests/test_forward_gpu.py -x -q --timeout 300 --timeout-method thread -k "prompt or prefill" > gpurun_out/fa5_tests.log 2>&1 || { tail -15 gpurun_out/fa5_tests.log; exit 1; }
tail -1 gpurun_out/fa5_tests.log
bash tools/exp_fa4.sh
