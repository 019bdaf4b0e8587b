export TMPDIR=/tmp
ARGS="--pos0 3800" LIBS="base ns32 ns32b2" WL="mistral-7b-f16 mistral-7b-f8" ROUNDS=2 bash tools/gpu_step.sh ab6 600 bash tools/abn.sh && \
LIBS="base ns32" WL="mistral-7b-f16" ROUNDS=1 bash tools/gpu_step.sh ab6s 300 bash tools/abn.sh && \
XALM_HIP_LIB=xalm_amd/lib/var_ns32.so bash tools/gpu_step.sh trns 200 python3 tools/aw_trace.py --pos0 3800
