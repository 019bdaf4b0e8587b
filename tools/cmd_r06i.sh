export TMPDIR=/tmp
XALM_ERR_LOG=gpurun_out/err_log.json XALM_PARITY_OUT=gpurun_out/parity_full.jsonl bash tools/gpu_step.sh pytest_gpu 1100 python3 -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -rs
