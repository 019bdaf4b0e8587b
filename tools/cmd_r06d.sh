export TMPDIR=/tmp
bash tools/gpu_step.sh t4 900 python3 -u -m pytest tests/test_regimes_gpu.py tests/test_forward_gpu.py tests/test_gq_gpu.py -x -q --timeout 300 --timeout-method thread && \
bash tools/gpu_step.sh tr4k 200 python3 tools/aw_trace.py --pos0 3800 && \
ARGS="--pos0 3800" LIBS="m4 m16" WL="mistral-7b-f16 mistral-7b-f8" ROUNDS=2 bash tools/gpu_step.sh ab3 600 bash tools/abn.sh && \
LIBS="m4 m16" WL="mistral-7b-f16" ROUNDS=1 bash tools/gpu_step.sh ab3s 300 bash tools/abn.sh && \
LIBS="q4old q4new" WL="mistral-7b-q4_0" ROUNDS=2 bash tools/gpu_step.sh ab4 600 bash tools/abn.sh
