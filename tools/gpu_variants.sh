#!/bin/bash
# kernel traces of the bench for the default library and variant builds (variants/<name>,
# loaded through MMAD_LIB_PATH); prints the lines of the step table matching a pattern
#   gpurun -- bash tools/gpu_variants.sh <tag> <grep pattern> <variant> ...
TAG=$1; PAT=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base "$@"; do
  L=""
  if [ $v != base ]; then L="MMAD_LIB_PATH=$GRAFT_REPO_ROOT/variants/$v/libmmad_hip.so"; fi
  timeout -k 10 200 env $L MMAD_X=1 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $OUT/prof_$v.log 2>&1 || { echo "$v failed"; tail -3 $OUT/prof_$v.log; exit 1; }
  python3 tools/prof_summary.py stepavg $OUT/prof_$v > $OUT/step_$v.txt 2>&1
  echo "== $v: $(head -1 $OUT/step_$v.txt)"; grep -E "$PAT" $OUT/step_$v.txt | cut -c1-80
done
echo session done
