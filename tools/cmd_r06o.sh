export TMPDIR=/tmp
bash tools/gpu_step.sh t8 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_regimes_gpu.py -x -q --timeout 300 --timeout-method thread -k "attention or mha or ring or long or 32k or sink" && \
STEPS=64 LIBS="base ring" WL="mistral-7b-f16-32k" ROUNDS=2 bash tools/gpu_step.sh ab12 600 bash tools/abn.sh
