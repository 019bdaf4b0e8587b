export TMPDIR=/tmp
LIBS="base zz" ROUNDS=3 bash tools/gpu_step.sh pfab1 600 bash tools/pf_ab.sh && \
XALM_HIP_LIB=xalm_amd/lib/var_zz.so bash tools/gpu_step.sh pfzz 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pfzz -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 5 --prefill-tokens 2048
