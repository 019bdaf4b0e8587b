export TMPDIR=/tmp
bash tools/gpu_step.sh t3 600 python3 -u -m pytest tests/test_gq_gpu.py tests/test_regimes_gpu.py tests/test_forward_gpu.py -x -q --timeout 200 --timeout-method thread -k "gq or prompt_attention or long_history or short_prompt or batched_prefill" && \
bash tools/gpu_step.sh tr4k 200 python3 tools/aw_trace.py --pos0 3800 && \
bash tools/gpu_step.sh tr0 200 python3 tools/aw_trace.py && \
bash tools/gpu_step.sh pr4k 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pr4k -o run --output-format csv -- python3 bench.py --pos0 3800 --steps 256 --warmup 8 --no-cpu-baseline --prefill-tokens 0 --kernel-iters 20 && \
LIBS="q4old q4new" WL="mistral-7b-q4_0" ROUNDS=3 bash tools/gpu_step.sh ab2 600 bash tools/abn.sh
