#!/bin/bash
# One GPU-box session: the new full-size oracle tests (verbose, printed errors), then the
# whole -m gpu suite.  A pytest exit of 0 or 1 (tests ran; some may have failed) lets the
# next step run; any other status (timeout 124/137, abort, segfault) ends the session.
#   gpurun --timeout 1100 -- bash tools/gpu_session.sh <tag> [pytest -k expr]
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {    # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step fullsize 300 python -u -m pytest tests/test_fullsize_oracle_gpu.py -v -s --timeout 240 --timeout-method thread
step suite 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --ignore=tests/test_fullsize_oracle_gpu.py
grep -E "FAILED|ERROR" $OUT/suite.log | head -20
echo session done
