#!/bin/bash
# kernel-trace durations + two SQ counter passes for the kernels of tools/probe_op.py --op OP
#   gpurun -- bash tools/gpu_pmc_op.sh <tag> <op> <kernel-substring> ...
TAG=$1; OP=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/probe_op.py --op $OP > $OUT/kt.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVES -d $OUT/a -o run --output-format csv -- python3 tools/probe_op.py --op $OP > $OUT/a.log 2>&1 || { echo "pmc a failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/b -o run --output-format csv -- python3 tools/probe_op.py --op $OP > $OUT/b.log 2>&1 || { echo "pmc b failed"; exit 1; }
python3 - $OUT "$@" <<'PY' | tee $OUT/pmc.txt
import csv, sys, collections
d, keys = sys.argv[1], sys.argv[2:]
for key in keys:
    v = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f"{d}/kt/run_kernel_trace.csv")) if key in r["Kernel_Name"])
    print(f"== {key}: duration_us n={len(v)} median={v[len(v)//2]/1e3:.1f}" if v else f"== {key}: none")
    k = collections.defaultdict(list)
    for sub in ("a", "b"):
        for r in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
            if key in r["Kernel_Name"]: k[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, vv in sorted(k.items()): print(f"   {c:28s} {sorted(vv)[len(vv)//2]:.4g}")
PY
echo session done
