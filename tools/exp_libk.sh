#!/bin/bash
# isolated kernel times of one probe layer/op, in-tree library vs a variant build:
#   bash tools/exp_libk.sh <varlib name> <layer> <op> [<layer> <op> ...]
set -o pipefail
N=$1; shift
OUT=gpurun_out/libk_$N
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
while [ $# -ge 2 ]; do
  L=$1; OP=$2; shift 2
  for X in tree $N; do
    if [ $X = tree ]; then LP=""; else LP=$PWD/varlib/$N/libmmad_hip.so; fi
    MMAD_LIB_PATH=$LP timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$L$OP$X -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP --reps 10 > $OUT/$L$OP$X.log 2>&1 || exit 1
    echo "== $L $OP $X"
    python tools/prof_summary.py stats $OUT/$L$OP$X 4
  done
done
