set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/attn_bench 32768 > gpurun_out/attn_bench_32k.txt 2>&1 || exit 1
cat gpurun_out/attn_bench_32k.txt
timeout -k 10 60 ./tools/attn_bench 4096 > gpurun_out/attn_bench_4k.txt 2>&1 || exit 1
head -5 gpurun_out/attn_bench_4k.txt
timeout -k 10 400 python -u -m pytest tests/test_forward_gpu.py -x -q --timeout 200 --timeout-method thread -k "long_context or multi_split or ring_buffer or forward_matches_oracle or prefill_matches" > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload mistral-7b-f16-32k --steps 64 --no-cpu-baseline --kernel-iters 20 > gpurun_out/bench32k.txt 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench32k.txt').read().strip().splitlines()[-1]);print('32k tok/s',d['value'],'ms',d['ms_per_step'], d['kernels']['attention'])"
