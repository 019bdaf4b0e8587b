export TMPDIR=/tmp
bash tools/gpu_step.sh t6 900 python3 -u -m pytest tests/test_ops_gpu.py tests/test_gq_gpu.py tests/test_forward_gpu.py tests/test_regimes_gpu.py -x -q --timeout 300 --timeout-method thread
