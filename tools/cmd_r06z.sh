export TMPDIR=/tmp
bash tools/gpu_step.sh mb_tests 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_forward_gpu.py tests/test_regimes_gpu.py tests/test_ops_gpu.py && \
LIBS="base mb" WL="mistral-7b-f16" ROUNDS=3 ARGS="--pos0 3800" bash tools/gpu_step.sh mb_ab4k 900 bash tools/abn.sh && \
LIBS="base mb" WL="mistral-7b-f8" ROUNDS=2 ARGS="--pos0 3800" bash tools/gpu_step.sh mb_ab4k8 600 bash tools/abn.sh
