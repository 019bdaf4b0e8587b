#!/bin/bash
# PMC counters of the decode kernels of one workload (WL), bench.py with few steps; one pass per
# counter set (SQ <= 8, TA <= 2, GRBM <= 2 per pass).
set -u
cd "$(dirname "$0")/.."
WL=${WL:-mistral-7b-q4_0}
OUT=gpurun_out/dpmc_$WL
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD TA_BUSY_sum GRBM_COUNT"; do
    i=$((i+1))
    echo "== pass $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- \
        python3 bench.py --workload $WL --steps 8 --warmup 2 --no-cpu-baseline --kernel-iters 5 --prefill-tokens 0 > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 "$OUT/p$i.log"; exit $rc; fi
done
exit 0
