"""Per-kernel PMC summary of tools/pmc.sh passes -> JSON (bytes per dispatch).

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.  On gfx950 FETCH_SIZE
counts half of the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM), so the
read traffic is 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores and atomics.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pass_dir, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    # one or more pass directories (e.g. the f16 and the fp8 workload), merged per kernel name
    fetch, write = defaultdict(list), defaultdict(list)
    for out in sys.argv[1:]:
        for k, v in load(os.path.join(out, "FETCH_SIZE"), "FETCH_SIZE").items():
            fetch[k] += v
        for k, v in load(os.path.join(out, "WRITE_SIZE"), "WRITE_SIZE").items():
            write[k] += v
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        res[k] = {
            "dispatches": max(len(f), len(w)),
            "fetch_size_kib_avg": sum(f) / len(f) if f else None,
            "read_bytes_avg": 2 * 1024 * sum(f) / len(f) if f else None,
            "write_bytes_avg": 1024 * sum(w) / len(w) if w else None,
        }
    print(json.dumps({"correction": "read = 2 x FETCH_SIZE (gfx950), KiB -> bytes", "kernels": res}, indent=1))


if __name__ == "__main__":
    main()
