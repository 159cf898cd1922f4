#!/bin/bash
# one tree, one box: GPU tests, two bench lines, a kernel-trace summary of the bench
#   exp_one.sh TAG
set -e -o pipefail
T=${1:-one}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
tail -1 gpurun_out/$T/pytest.log
for i in 1 2; do
  timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T/b$i.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/$T/b$i.json'));print('vol/s', round(d['value'],1), 'ms', round(d['ms_per_step'],3))" | tee -a gpurun_out/$T/bench.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1
python tools/prof_summary.py step gpurun_out/$T/prof > gpurun_out/$T/step.txt
sort -n gpurun_out/$T/step.txt | tail -30
