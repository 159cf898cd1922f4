#!/bin/bash
# Round-3 third session: graph-mode DP test, plane-pair variant A/B (variant libraries under
# variants/, built beforehand with `python -m multimodal_alzheimer_amd._build --variant ...`),
# SQ counters of the layer4 / layer3 kernels, eager and one-rank RCCL bench lines.
TAG=${1:-r03c}
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
step tests 300 $PYT tests/test_graph_step_gpu.py tests/test_lattice_zp_gpu.py
for v in zp_late zp_early2; do
  step ab_$v 200 env MMAD_LIB_PATH=variants/$v/libmmad_hip.so python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
step ab_default 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step pmc_l4 200 bash tools/pmc_kernel.sh l4c2 fwd lattice_zp
step pmc_l3 200 bash tools/pmc_kernel.sh l3c2 fwd lattice8
step pmc_l4w 200 bash tools/pmc_kernel.sh l4c2 wgrad lattice_wgrad
step eager 200 python -u bench.py --eager --steps 20 --warmup 5 --no-cpu-baseline --no-roofline
step dp1 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --steps 20 --warmup 5 --no-roofline
step dp1eager 300 env MMAD_DP_SELFTEST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29572 bench.py --eager --steps 20 --warmup 5 --no-roofline
echo session done
