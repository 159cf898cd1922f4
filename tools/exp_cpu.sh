#!/bin/bash
set -e -o pipefail
T=${1:-cpu}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
timeout -k 10 120 python -u tools/cpu_bound.py > gpurun_out/$T/cpu.txt 2>&1
MMAD_DP_SELFTEST=1 timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$T/bench_dp1.json 2> gpurun_out/$T/bench_dp1.err
grep -v amdgpu.ids gpurun_out/$T/cpu.txt; echo "--- dp1 stdout:"; cat gpurun_out/$T/bench_dp1.json
