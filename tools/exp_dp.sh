#!/bin/bash
# RCCL gradient all-reduce path at N=1 (torchrun, MMAD_DP_SELFTEST) vs the plain N=1 bench
set -e -o pipefail
T=${1:-dp}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T/b1.json 2> gpurun_out/$T/b1.err
MMAD_DP_SELFTEST=1 timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T/dp1.json 2> gpurun_out/$T/dp1.err
for f in b1 dp1; do python -c "import json;d=json.load(open('gpurun_out/$T/$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3))"; done
