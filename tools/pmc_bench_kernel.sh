#!/bin/bash
# HBM bytes (FETCH_SIZE, WRITE_SIZE: two passes) of one kernel of the bench's graph replays:
#   bash tools/pmc_bench_kernel.sh <tag> <kernel-name-substring>
set -o pipefail
TAG=$1; K=$2
OUT=gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/$c -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/$c.log 2>&1 || exit 1
done
python3 - $OUT $K <<'PY'
import csv, sys, collections, glob
d, key = sys.argv[1], sys.argv[2]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = collections.defaultdict(float)
    for f in glob.glob(f"{d}/{c}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                v[r["Dispatch_Id"]] += float(r["Counter_Value"])
    vals = sorted(v.values())
    print(c, "dispatches", len(vals), "KiB per dispatch (median)", vals[len(vals) // 2] if vals else None)
PY
