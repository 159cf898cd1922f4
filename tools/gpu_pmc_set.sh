#!/bin/bash
# SQ counters (tools/pmc_kernel.sh) + kernel-trace durations for a set of layer kernels
#   gpurun -- bash tools/gpu_pmc_set.sh <tag> "layer:op:kernel-substring" ...
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
  IFS=: read L OP K <<< "$spec"
  echo "== $L $OP $K" | tee -a $OUT/pmc.txt
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt_$L$OP -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP $PROBE_ARGS > $OUT/kt_$L$OP.log 2>&1 || { echo "trace failed"; exit 1; }
  python3 - $OUT/kt_$L$OP $K <<'PY' | tee -a $OUT/pmc.txt
import csv, sys
d, key = sys.argv[1], sys.argv[2]
v = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")) if key in r["Kernel_Name"]]
v.sort()
print(f"   duration_us n={len(v)} median={v[len(v)//2]/1e3:.1f}" if v else "   no such kernel")
PY
  bash tools/pmc_kernel.sh $L $OP $K | tee -a $OUT/pmc.txt || { echo "pmc failed"; exit 1; }
done
echo session done
