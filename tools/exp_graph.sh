#!/bin/bash
# graph-replay step: parity test, then eager vs graph bench lines
set -e -o pipefail
T=${1:-graph}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_graph_step_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for m in "" "--graph" "" "--graph"; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $m > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err
  python -c "import json;d=json.load(open('gpurun_out/$T/b.json'));print('mode=$m', 'vol/s', round(d['value'],1), 'ms', round(d['ms_per_step'],3))" | tee -a gpurun_out/$T/bench.txt
done
