export TMPDIR=/tmp
mkdir -p gpurun_out/r06b
bash tools/gpu_step.sh r06b_bench 600 python3 bench.py && \
bash tools/gpu_step.sh r06b_bench_f8 600 python3 bench.py --workload mistral-7b-f8 && \
bash tools/gpu_step.sh r06b_bench_kv4k 300 python3 bench.py --pos0 3800 --prefill-tokens 0
