#!/bin/bash
# Round-3 session: diagnose the graph + after-replay all-reduce mismatch (tools/diag_after.py),
# the recalibrated bf16 full-size oracle test, the bench line with the shipped defaults
# (pipelined plane-pair lattice + z-walking layer1 conv; barrier-first wgrad / lattice8,
# rows pool kernel), and a kernel trace per lattice-wgrad build: default (barrier-first),
# variants/lwpipe (pipelined, z padding skipped), variants/lwpipe_noskip (pipelined).
TAG=${1:-r03f}
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
step diag 200 python -u tools/diag_after.py
cat $OUT/diag.log | grep -v "^\[W\|RCCL\|HIP version\|ROCm version\|Hostname\|Librccl" | head -40
step tests 400 $PYT -s tests/test_fullsize_oracle_gpu.py tests/test_fullsize_gpu.py tests/test_patchz_gpu.py "tests/test_kernels_gpu.py::test_bn_relu_maxpool_fused"
step bench 200 python -u bench.py --steps 20 --warmup 5
for v in default lwpipe lwpipe_noskip; do
  LIB=multimodal_alzheimer_amd/libmmad_hip.so
  if [ $v != default ]; then LIB=variants/$v/libmmad_hip.so; fi
  step prof_$v 200 env MMAD_LIB_PATH=$LIB rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  python3 tools/prof_summary.py stepavg $OUT/prof_$v > $OUT/step_$v.txt 2>&1; head -1 $OUT/step_$v.txt; grep -E "lattice_wgrad" $OUT/step_$v.txt | cut -c1-70
done
echo session done
