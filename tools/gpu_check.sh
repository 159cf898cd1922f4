#!/bin/bash
# A new kernel's check in one call: the named GPU tests, then a kernel trace of the bench
# (11-step average table) and a bench line.
#   gpurun -- bash tools/gpu_check.sh <tag> "<test files>" "<-k expression>" [VAR=value ...]
# Extra VAR=value arguments are exported for the trace and the bench (A/B switches).
TAG=${1:-chk}
SEL=$2
KX=$3
shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for kv in "$@"; do export "$kv"; done
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return $rc
}
if [ -n "$SEL" ]; then
  step tests 500 $PYT $SEL ${KX:+-k "$KX"} || { grep -E "^(FAILED|ERROR)|Error" $OUT/tests.log | head -20; exit 1; }
fi
step prof 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
python3 tools/prof_summary.py stepavg $OUT/prof > $OUT/step.txt 2>&1; cat $OUT/step.txt
step bench 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo session done
