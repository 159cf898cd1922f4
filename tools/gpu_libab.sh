#!/bin/bash
# kernel traces of the bench with several library builds (MMAD_LIB_PATH), same box, in order
#   gpurun -- bash tools/gpu_libab.sh <tag> <grep pattern> lib1.so lib2.so ...
TAG=$1; PAT=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for lib in "$@"; do
  i=$((i + 1))
  timeout -k 10 200 env MMAD_LIB_PATH=$lib rocprofv3 --kernel-trace --stats -d $OUT/prof_$i -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $OUT/prof_$i.log 2>&1 || { echo "$lib failed"; tail -3 $OUT/prof_$i.log; exit 1; }
  python3 tools/prof_summary.py stepavg $OUT/prof_$i > $OUT/step_$i.txt 2>&1
  echo "== $i $lib: $(head -1 $OUT/step_$i.txt)"; grep -E "$PAT" $OUT/step_$i.txt | cut -c1-80
done
echo session done
