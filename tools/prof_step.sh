#!/bin/bash
# rocprof kernel trace of a short bench run + per-step kernel table (one step, in order)
set -e -o pipefail
T=${1:-ps}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$T
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1
python3 tools/prof_summary.py stats gpurun_out/$T/prof 60
python3 tools/prof_summary.py step gpurun_out/$T/prof > gpurun_out/$T/step.txt
