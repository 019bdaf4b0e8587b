#!/bin/bash
# One GPU call = several steps, each under its own time limit; the first failing step ends the call.
#   bash tools/gpu_step.sh NAME LIMIT cmd...   (appends to gpurun_out/NAME.log)
set -u
name=$1 limit=$2
shift 2
mkdir -p gpurun_out
echo "== $name $(date +%T)"
timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc"
if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.log"; fi
exit $rc
