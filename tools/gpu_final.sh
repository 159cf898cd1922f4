#!/bin/bash
# Round-end validation of HEAD in one call: the whole -m gpu suite as the driver runs it,
# smoke(), the config-2 bench line (roofline + cpu_baseline), rocprofv3 kernel stats + the
# 11-step kernel table, the PMC traffic passes of layer4.0.conv2's forward and weight
# gradient, the one-rank
# RCCL bench in the N > 1 launch mode.  Each GPU step has its own limit; a fault ends it.
TAG=${1:-r03final}
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
step suite 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 240 python -u bench.py --steps 20 --warmup 5
step prof 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline
python3 tools/prof_summary.py stats $OUT/prof 40 > $OUT/stats.txt 2>&1
python3 tools/prof_summary.py stepavg $OUT/prof > $OUT/step.txt 2>&1
head -1 $OUT/step.txt
step pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/probe_dominant.py
step pmc_write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/probe_dominant.py
python3 tools/prof_summary.py traffic $OUT/pmc_fetch $OUT/pmc_write > $OUT/traffic.json 2>&1; cat $OUT/traffic.json | head -5
step pmc_wfetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_wfetch -o run --output-format csv -- python3 tools/probe_dominant.py --op wgrad
step pmc_wwrite 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_wwrite -o run --output-format csv -- python3 tools/probe_dominant.py --op wgrad
python3 tools/prof_summary.py traffic $OUT/pmc_wfetch $OUT/pmc_wwrite wgrad > $OUT/traffic_wgrad.json 2>&1; cat $OUT/traffic_wgrad.json | head -5
step dp1 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --steps 20 --warmup 5 --no-roofline --no-cpu-baseline
echo session done
