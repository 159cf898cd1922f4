#!/bin/bash
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lattice5_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload three --steps 6 --warmup 2 > $OUT/t_l5_$i.json 2> $OUT/t_l5_$i.err || exit 1
  MMAD_LATTICE5=0 timeout -k 10 300 python -u bench.py --workload three --steps 6 --warmup 2 > $OUT/t_off_$i.json 2> $OUT/t_off_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload three --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || exit 1
python3 tools/prof_summary.py stats $OUT/prof > $OUT/stats.txt 2>&1
for f in $OUT/*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value'], 2), round(d['ms_per_step'], 3))"
done
head -20 $OUT/stats.txt
echo session done
