export TMPDIR=/tmp
XALM_HIP_LIB=xalm_amd/lib/var_gw2.so bash tools/gpu_step.sh t7 600 python3 -u -m pytest tests/test_gq_gpu.py -x -q --timeout 300 --timeout-method thread && \
LIBS="base gw2" WL="mistral-7b-q8_0 mistral-7b-q4_0" ROUNDS=2 bash tools/gpu_step.sh ab10 600 bash tools/abn.sh
