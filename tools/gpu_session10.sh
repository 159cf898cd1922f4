#!/bin/bash
# lattice wgrad with compile-time z skipping (LW_TZ=1, default) against the zero-block form
# (variants/lwtz0): layer tests, then a kernel trace per build
TAG=${1:-r03p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step tests 300 $PYT tests/test_fullsize_gpu.py tests/test_mni_geometry_gpu.py tests/test_twin_gpu.py tests/test_fullsize_oracle_gpu.py
for v in default lwtz0; do
  LIB=multimodal_alzheimer_amd/libmmad_hip.so
  if [ $v != default ]; then LIB=variants/$v/libmmad_hip.so; fi
  step prof_$v 200 env MMAD_LIB_PATH=$LIB rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  python3 tools/prof_summary.py stepavg $OUT/prof_$v > $OUT/step_$v.txt 2>&1; head -1 $OUT/step_$v.txt; grep -E "lattice_wgrad" $OUT/step_$v.txt | cut -c1-70
done
step bench 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo session done
