#!/bin/bash
# Kernel stats + one step's kernel table of the bench (no tests, no PMC).
#   gpurun -- bash tools/prof_step.sh <tag>
set -e -o pipefail
OUT=gpurun_out/${1:-step}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
python3 tools/prof_summary.py stats $OUT/prof 40 > $OUT/stats.txt
python3 tools/prof_summary.py step $OUT/prof > $OUT/step.txt
python3 tools/step_breakdown.py $OUT/step.txt
