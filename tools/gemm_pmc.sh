#!/bin/bash
# PMC counters of the prompt GEMM (tools/gemm_bench, one variant, W1/W3 shape at 2048 tokens).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/gpmc
mkdir -p "$OUT"
export TMPDIR=/tmp GB_NOBLAS=1 GB_SHAPE=${GB_SHAPE:-w13} GB_VAR=${GB_VAR:-0}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS GRBM_COUNT" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    echo "== pass $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- tools/gemm_bench 2048 > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    [ $rc -ne 0 ] && { tail -3 "$OUT/p$i.log"; exit $rc; }
done
