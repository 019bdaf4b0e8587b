export TMPDIR=/tmp
bash tools/gpu_step.sh m5_tests 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_forward_gpu.py -k "prefill" && \
for r in 1 2 3; do for w in mistral-7b-f16 mistral-7b-f8; do for m in 1 5; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 8 --warmup 2 --no-cpu-baseline --kernel-iters 5 --prefill-mode $m > gpurun_out/pfm.json 2> gpurun_out/pfm.err || { echo FAILED; tail -5 gpurun_out/pfm.err; exit 1; }
  python3 -c "
import json; d = json.load(open('gpurun_out/pfm.json')); p = d['prefill']
print('$w mode $m', p.get('tok_s'), p.get('ms'), (p.get('perplexity') or {}).get('tok_s'), flush=True)" >> gpurun_out/m5_ab.log
done; done; done
cat gpurun_out/m5_ab.log
