export TMPDIR=/tmp
ARGS="--pos0 3800" LIBS="base b1 b2 c1 c0" WL="mistral-7b-f16" ROUNDS=2 bash tools/gpu_step.sh ab5 600 bash tools/abn.sh && \
LIBS="base b2 c1" WL="mistral-7b-f16" ROUNDS=1 bash tools/gpu_step.sh ab5s 300 bash tools/abn.sh && \
XALM_HIP_LIB=xalm_amd/lib/var_b2.so bash tools/gpu_step.sh trb2 200 python3 tools/aw_trace.py --pos0 3800 && \
XALM_HIP_LIB=xalm_amd/lib/var_c1.so bash tools/gpu_step.sh trc1 200 python3 tools/aw_trace.py --pos0 3800
