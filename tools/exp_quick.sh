#!/bin/bash
# quick perf check: per-conv table + bench line (no tests)
set -e -o pipefail
T=${1:-q}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
timeout -k 10 120 python -u tools/bench_conv.py --no-miopen > gpurun_out/$T/conv.txt 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
cat gpurun_out/$T/conv.txt gpurun_out/$T/bench.json
