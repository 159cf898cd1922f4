#!/bin/bash
# tests given as $2.. (pytest node ids), then the config-5 bench (eager and graphed), the
# config-2 bench and a config-5 kernel trace; results under gpurun_out/$1
#   gpurun -- bash tools/gpu_round.sh TAG tests/test_a.py tests/test_b.py ...
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
timeout -k 10 300 python -u bench.py --workload three --steps 6 --warmup 2 > $OUT/three.json 2> $OUT/three.err || { tail -5 $OUT/three.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload three --steps 6 --warmup 2 --graph > $OUT/three_graph.json 2> $OUT/three_graph.err || tail -5 $OUT/three_graph.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/c2.json 2> $OUT/c2.err || { tail -5 $OUT/c2.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload three --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || exit 1
python3 tools/step_kernels.py $OUT/prof/run_kernel_trace.csv 40 > $OUT/step.txt 2>&1
for f in $OUT/*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value'], 2), round(d['ms_per_step'], 3), d.get('host_issue_ms_per_step'))" || true
done
head -24 $OUT/step.txt
echo session done
