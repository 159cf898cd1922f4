#!/bin/bash
# lattice8 with one plane row per wave (MMAD_L8_ROWS=1, default) against two (=2): layer
# tests, kernel traces, bench; the N > 1 graph mode with mid-replay bucket events (default)
# and without (--no-overlap) at one RCCL rank
TAG=${1:-r03r}
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
step tests 400 $PYT tests/test_fullsize_gpu.py tests/test_mni_geometry_gpu.py tests/test_fullsize_oracle_gpu.py tests/test_model_parity_gpu.py tests/test_graph_step_gpu.py
for v in rows1 rows2; do
  R=1; if [ $v = rows2 ]; then R=2; fi
  step prof_$v 200 env MMAD_L8_ROWS=$R rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  python3 tools/prof_summary.py stepavg $OUT/prof_$v > $OUT/step_$v.txt 2>&1; head -1 $OUT/step_$v.txt; grep -E "lattice8" $OUT/step_$v.txt | cut -c1-70
done
step bench 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step dp1 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --steps 20 --warmup 5 --no-roofline --no-cpu-baseline
step dp1noov 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29572 bench.py --no-overlap --steps 20 --warmup 5 --no-roofline --no-cpu-baseline
echo session done
