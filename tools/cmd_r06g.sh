export TMPDIR=/tmp
bash tools/gpu_step.sh t5 600 python3 -u -m pytest tests/test_gq_gpu.py tests/test_forward_gpu.py -x -q --timeout 300 --timeout-method thread && \
bash tools/gpu_step.sh gb 300 tools/gemm_bench 2048
