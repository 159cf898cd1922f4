#!/bin/bash
# replay determinism of a forward + backward-only graph, and the graph + after-replay
# all-reduce mode against eager steps (tools/diag_replay.py, tools/diag_after.py)
TAG=${1:-r03m}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in none adam; do
  timeout -k 10 120 python -u tools/diag_replay.py $s > $OUT/replay_$s.log 2>&1
  rc=$?
  echo "replay $s rc=$rc"; grep "^$s" $OUT/replay_$s.log | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 $OUT/replay_$s.log; exit $rc; fi
done
for s in after plainnoopt; do
  timeout -k 10 120 python -u tools/diag_after.py $s > $OUT/diag_$s.log 2>&1
  rc=$?
  echo "diag $s rc=$rc"; grep "^$s " $OUT/diag_$s.log | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 $OUT/diag_$s.log; exit $rc; fi
done
