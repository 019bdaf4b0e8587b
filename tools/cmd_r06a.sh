bash tools/gpu_step.sh t1 500 python3 -u -m pytest tests/test_regimes_gpu.py -x -v --timeout 200 --timeout-method thread -k "prompt_attention or long_history or short_prompt" && \
bash tools/gpu_step.sh b32k 400 python3 bench.py --workload mistral-7b-f16-32k --steps 32 --warmup 4 --no-cpu-baseline --kernel-iters 20 && \
bash tools/gpu_step.sh kv4k 300 python3 bench.py --pos0 3808 --no-cpu-baseline --prefill-tokens 0 && \
LIBS="base hold first4 first2" WL="mistral-7b-f16 mistral-7b-f8" ROUNDS=2 bash tools/gpu_step.sh ab1 900 bash tools/abn.sh
