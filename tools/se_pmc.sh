#!/bin/bash
# I-cache and wave-state counters for the stream kernel vs the graph engine (one rocprofv3 pass each).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for e in 2 0; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmc/e$e -o run --output-format csv -- python3 tools/se_decode.py --engine $e --tokens 8 > gpurun_out/pmc/e$e.log 2>&1
  rc=$?
  echo "engine $e rc=$rc"; tail -2 gpurun_out/pmc/e$e.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 - <<'PY'
import csv, glob, collections
for e in (2, 0):
    fs = glob.glob(f"gpurun_out/pmc/e{e}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.Counter())
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")[:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    print("engine", e)
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQC_ICACHE_MISSES", 0))[:6]:
        h, m = v.get("SQC_ICACHE_HITS", 0), v.get("SQC_ICACHE_MISSES", 0)
        print(f"  {k:60s} icache miss {m:12.0f} hit {h:14.0f} miss rate {m / max(1, h + m):.4f}  valu {v.get('SQ_INSTS_VALU', 0):.3g}")
PY
