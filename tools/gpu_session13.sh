#!/bin/bash
# whole -m gpu suite; igemm A/B (ring depth 3, big tiles on the K = 256 shortcut as before)
# by kernel traces; bench; the N > 1 graph mode with mid-replay bucket events (C-ABI external
# events) and without, at one RCCL rank
TAG=${1:-r03s}
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
step tests 400 $PYT -m gpu tests
for v in base nst3 oldbig; do
  E=""
  if [ $v = nst3 ]; then E="MMAD_IGEMM_NST=3"; fi
  if [ $v = oldbig ]; then E="MMAD_IGEMM_BIG_MINK=0"; fi
  step prof_$v 200 env $E MMAD_X=1 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  python3 tools/prof_summary.py stepavg $OUT/prof_$v > $OUT/step_$v.txt 2>&1; head -1 $OUT/step_$v.txt; grep -E "igemm" $OUT/step_$v.txt | cut -c1-80
done
step bench 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step dp1 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --steps 20 --warmup 5 --no-roofline --no-cpu-baseline
step dp1noov 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29572 bench.py --no-overlap --steps 20 --warmup 5 --no-roofline --no-cpu-baseline
echo session done
