#!/bin/bash
# multi-rank rehearsal of the driver's scaling launch on a one-GPU box: N replicas under
# torch.distributed.run, all on device 0 (they share its HBM, so per-rank rates drop; this checks
# the launch, the barriers, the max-over-ranks timing and the aggregate line, not scaling)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp XALM_BENCH_DEVICE=0
N=${N:-2}
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus $N --steps 32 --warmup 4 --kernel-iters 5 --prefill-tokens 256 \
    > gpurun_out/rehearse_$N.log 2>&1
rc=$?
tail -2 gpurun_out/rehearse_$N.log | cut -c1-600
exit $rc
