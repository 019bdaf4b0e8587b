export TMPDIR=/tmp
STEPS=64 LIBS="base wpf" WL="mistral-7b-f16-32k" ROUNDS=2 bash tools/gpu_step.sh ab7 600 bash tools/abn.sh && \
ARGS="--pos0 3800" LIBS="base wpf" WL="mistral-7b-f16" ROUNDS=2 bash tools/gpu_step.sh ab7b 400 bash tools/abn.sh && \
bash tools/gpu_step.sh t5 600 python3 -u -m pytest tests/test_gq_gpu.py tests/test_forward_gpu.py -x -q --timeout 300 --timeout-method thread && \
bash tools/gpu_step.sh gb 300 tools/gemm_bench 2048
