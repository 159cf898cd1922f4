#!/bin/bash
# L2 hit-rate pass over one conv kernel:  bash tools/pmc_l2.sh <layer> <op> <tag>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$1; OP=$2; T=${3:-pmc}
D=gpurun_out/$T/${L}_${OP}_l2
mkdir -p $D
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $D/a -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP > $D/a.log 2>&1
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
PY
