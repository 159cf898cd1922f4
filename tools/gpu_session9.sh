#!/bin/bash
# Round-3 validation: the whole -m gpu suite as the driver runs it, smoke(), the config-2
# bench line, the one-rank RCCL bench in the N > 1 launch mode (graph + after-replay
# all-reduce) and in eager mode.
TAG=${1:-r03o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 200 python -u bench.py --steps 20 --warmup 5
step dp1 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --steps 20 --warmup 5 --no-roofline --no-cpu-baseline
step dp1eager 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29572 bench.py --eager --steps 20 --warmup 5 --no-roofline --no-cpu-baseline
echo session done
