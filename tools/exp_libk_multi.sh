#!/bin/bash
# isolated kernel time of one probe layer/op for several variant builds:
#   bash tools/exp_libk_multi.sh <layer> <op> <kernel-substring> <varlib name>...   ("tree" = in-tree)
set -o pipefail
L=$1; OP=$2; K=$3; shift 3
OUT=gpurun_out/libkm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for N in "$@"; do
  if [ $N = tree ]; then LP=""; else LP=$PWD/varlib/$N/libmmad_hip.so; fi
  MMAD_LIB_PATH=$LP timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$L$OP$N -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP --reps 10 > $OUT/$L$OP$N.log 2>&1 || exit 1
  echo "$N $(python tools/prof_summary.py stats $OUT/$L$OP$N 20 | grep "$K" | awk '{print $4}')"
done
