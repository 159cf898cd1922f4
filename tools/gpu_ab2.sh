#!/bin/bash
# Same-box A/B of the config-2 bench: the in-tree library against variants/$2 (MMAD_LIB_PATH),
# interleaved three times, after the tests given as $3..
#   gpurun -- bash tools/gpu_ab2.sh TAG VARIANT tests/test_a.py ...
TAG=$1; V=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
VL=$GRAFT_REPO_ROOT/variants/$V/libmmad_hip.so
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/new_$i.json 2> $OUT/new_$i.err || { tail -5 $OUT/new_$i.err; exit 1; }
  MMAD_LIB_PATH=$VL timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/old_$i.json 2> $OUT/old_$i.err || { tail -5 $OUT/old_$i.err; exit 1; }
done
for f in $OUT/*.json; do
  python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value'], 2), round(d['ms_per_step'], 4))" || true
done
echo session done
