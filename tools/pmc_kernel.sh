#!/bin/bash
# SQ counters of one kernel of tools/probe_kernel.py:  bash tools/pmc_kernel.sh <layer> <op> <name-substring>
set -o pipefail
L=$1; OP=$2; K=$3
OUT=gpurun_out/pmc1_$L$OP
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/a -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP $PROBE_ARGS > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/b -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP $PROBE_ARGS > $OUT/b.log 2>&1 || exit 1
python3 - $OUT $K <<'PY'
import csv, sys, collections
d, key = sys.argv[1], sys.argv[2]
k = collections.defaultdict(list)
for sub in ("a", "b"):
    for r in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
        if key in r["Kernel_Name"]: k[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(k.items()): print(f"   {c:28s} {sum(v)/len(v):.4g}")
PY
