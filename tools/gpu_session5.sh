#!/bin/bash
# Round-3 session: the pipelined stage loops (plane-pair lattice, lattice wgrad, lattice8)
# against the layer-level fp32 references, the plane-pair equality test, the full-size
# oracle fixtures and the graph-mode tests, then a kernel
# trace of 10 bench steps per build: default (all pipelined), variants/nopipe (all three
# barrier-first), variants/lw0, variants/l80 (one kernel reverted each), MMAD_PATCHZ=0 (per-box layer1 conv); PMC traffic of the dominant kernel.
TAG=${1:-r03e}
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
step tests 500 $PYT -s tests/test_patchz_gpu.py tests/test_lattice_zp_gpu.py tests/test_fullsize_gpu.py tests/test_mni_geometry_gpu.py tests/test_fullsize_oracle_gpu.py tests/test_graph_step_gpu.py "tests/test_kernels_gpu.py::test_bnpool_run_kernel_matches_rows_kernel" "tests/test_kernels_gpu.py::test_bn_relu_maxpool_fused" tests/test_twin_gpu.py
step bench 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
for v in default nopipe patchz0; do
  LIB=multimodal_alzheimer_amd/libmmad_hip.so; EXTRA=MMAD_NONE=0
  if [ $v = nopipe ]; then LIB=variants/$v/libmmad_hip.so; fi
  if [ $v = patchz0 ]; then EXTRA=MMAD_PATCHZ=0; fi
  step prof_$v 200 env MMAD_LIB_PATH=$LIB $EXTRA rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  python3 tools/prof_summary.py stepavg $OUT/prof_$v > $OUT/step_$v.txt 2>&1; head -1 $OUT/step_$v.txt; grep -E "lattice|patch|bnpool" $OUT/step_$v.txt | cut -c1-70
done
step fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/probe_dominant.py
step write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/probe_dominant.py
python3 tools/prof_summary.py traffic $OUT/pmc_fetch $OUT/pmc_write > $OUT/traffic.json
head -8 $OUT/traffic.json
echo session done
