#!/bin/bash
# One GPU-box session: the new kernel's equality test, the graph-capture regression test, the
# full-size oracle tests, the whole -m gpu suite, then bench lines (plane-pair lattice on / off).
# A pytest exit of 0 or 1 (tests ran; some may have failed) lets the next step run; any other
# status (timeout 124/137, abort, segfault) ends the session.
#   gpurun --timeout 1100 -- bash tools/gpu_session.sh <tag>
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
step() {    # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step zp 240 $PYT tests/test_lattice_zp_gpu.py
step capture 200 $PYT tests/test_graph_step_gpu.py -k capture_after_eager
step fullsize 300 $PYT -s tests/test_fullsize_oracle_gpu.py
step suite 700 $PYT tests -m gpu --ignore=tests/test_fullsize_oracle_gpu.py --ignore=tests/test_lattice_zp_gpu.py
grep -E "FAILED|ERROR" $OUT/suite.log | head -20
grep -c "AccumulateGrad" $OUT/*.log
step bench1 240 python -u bench.py --steps 20 --warmup 5
step bench0 240 env MMAD_LATTICE_ZP=0 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step benchpw 240 env MMAD_PW_GEMM=0 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline
python3 tools/prof_summary.py stats $OUT/prof 40 > $OUT/stats.txt
python3 tools/prof_summary.py step $OUT/prof > $OUT/step.txt
python3 tools/step_breakdown.py $OUT/step.txt > $OUT/breakdown.txt
cat $OUT/breakdown.txt
echo session done
