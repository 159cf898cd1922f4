#!/bin/bash
# interleaved bench A/B of an env switch:  bash tools/exp_ab.sh VAR valA valB [reps]
set -o pipefail
V=$1; A=$2; B=$3; R=${4:-2}
OUT=gpurun_out/ab_$V
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in $(seq $R); do
  for X in $A $B; do
    env "$V=$X" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_$X.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b_$X.json'));print('$V=$X', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms']*1e3,1))"
  done
done
