#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprof kernel stats, PMC traffic passes.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh <tag> [skip_tests]
# Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "${2:-}" != "skip_tests" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1
  echo "pytest gpu ok"
fi
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
echo "rocprof stats ok"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv \
  -- python3 tools/probe_dominant.py > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv \
  -- python3 tools/probe_dominant.py > $OUT/pmc_write.log 2>&1
echo "pmc ok"
python3 tools/prof_summary.py traffic $OUT/pmc_fetch $OUT/pmc_write > $OUT/traffic.json
python3 tools/prof_summary.py stats $OUT/prof 40 > $OUT/stats.txt
python3 tools/prof_summary.py step $OUT/prof > $OUT/step.txt
echo "summaries ok"
