#!/bin/bash
# diagnose the graph + after-replay all-reduce gradient mismatch (tools/diag_after.py)
TAG=${1:-r03g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in insidenoopt plainnoopt; do
  timeout -k 10 120 python -u tools/diag_after.py $s > $OUT/diag_$s.log 2>&1
  rc=$?
  echo "diag $s rc=$rc"
  grep "^$s " $OUT/diag_$s.log | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 $OUT/diag_$s.log; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
