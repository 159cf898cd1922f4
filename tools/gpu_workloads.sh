#!/bin/bash
# secondary bench lines: BASELINE config 3 (PET+MRI fusion), config 5 (three modalities,
# 160^3) and config 2 on the reference's MNI geometry
TAG=${1:-r03wl}
EXTRA=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in "fusion" "three" "mni"; do
  if [ $w = mni ]; then A="--size mni"; else A="--workload $w"; fi
  timeout -k 10 300 python -u bench.py $A $EXTRA --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $OUT/$w.json 2> $OUT/$w.err
  rc=$?; echo "$w rc=$rc"; grep '^{' $OUT/$w.json | cut -c1-400
  if [ $rc -ne 0 ]; then tail -3 $OUT/$w.err; exit $rc; fi
done
echo session done
