export TMPDIR=/tmp
bash tools/gpu_step.sh t2 500 python3 -u -m pytest tests/test_regimes_gpu.py -x -v --timeout 200 --timeout-method thread -k "prompt_attention or long_history or short_prompt" && \
bash tools/gpu_step.sh sp1 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sp1 -o run --output-format csv -- python3 tools/short_pass.py 1 && \
bash tools/gpu_step.sh sp32 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sp32 -o run --output-format csv -- python3 tools/short_pass.py 32 && \
bash tools/gpu_step.sh sp256 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sp256 -o run --output-format csv -- python3 tools/short_pass.py 256 && \
bash tools/gpu_step.sh kv4k 300 python3 bench.py --pos0 3800 --no-cpu-baseline --prefill-tokens 0 && \
LIBS="base hold first4 first2" WL="mistral-7b-f16 mistral-7b-f8" ROUNDS=2 bash tools/gpu_step.sh ab1 900 bash tools/abn.sh
