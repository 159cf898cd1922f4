#!/bin/bash
# interleaved bench A/B of the in-tree library against a variant build:
#   bash tools/exp_lib_ab.sh <varlib name> [reps]     (varlib/<name>/libmmad_hip.so)
set -o pipefail
N=$1; R=${2:-3}
OUT=gpurun_out/ablib_$N
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in $(seq $R); do
  for X in base $N; do
    if [ $X = base ]; then LP=""; else LP=$PWD/varlib/$N/libmmad_hip.so; fi
    MMAD_LIB_PATH=$LP timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_$X.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b_$X.json'));print('$X', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
