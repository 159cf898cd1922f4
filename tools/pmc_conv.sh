#!/bin/bash
# SQ counter pass over one conv kernel:  bash tools/pmc_conv.sh <layer> <op> <tag>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$1; OP=$2; T=${3:-pmc}
D=gpurun_out/$T/${L}_${OP}
mkdir -p $D
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $D/a -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP > $D/a.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP > $D/t.log 2>&1
python3 - "$D" <<'PY'
import csv, sys, collections
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/a/run_counter_collection.csv")))
k = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in k.items():
    print(name)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):.4g}")
st = list(csv.DictReader(open(f"{d}/t/run_kernel_stats.csv")))
for r in st:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']}  {r['Name'][:80]}")
PY
