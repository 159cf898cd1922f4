#!/bin/bash
# kernel traces of the bench under several values of one environment switch
#   gpurun -- bash tools/gpu_envab.sh <tag> <grep pattern> VAR val1 val2 ...
TAG=$1; PAT=$2; VAR=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  timeout -k 10 200 env $VAR=$v rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $OUT/prof_$v.log 2>&1 || { echo "$v failed"; tail -3 $OUT/prof_$v.log; exit 1; }
  python3 tools/prof_summary.py stepavg $OUT/prof_$v > $OUT/step_$v.txt 2>&1
  echo "== $VAR=$v: $(head -1 $OUT/step_$v.txt)"; grep -E "$PAT" $OUT/step_$v.txt | cut -c1-80
done
echo session done
