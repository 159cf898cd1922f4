#!/bin/bash
# One-GPU RCCL self-test: the GPU DP parity test, bench lines alternating the in-place bucket
# slots (MMAD_DP_GRAD_SLOTS), then a kernel trace with the default.
set -e -o pipefail
O=gpurun_out/${1:-dpab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "allreduce or data_parallel or GradAllReduce or dp" > $O/pytest_dp.log 2>&1
tail -1 $O/pytest_dp.log
port=29580
for rep in 1 2; do
  for v in 1 0; do
    port=$((port+1))
    RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port MMAD_DP_SELFTEST=1 \
      MMAD_DP_GRAD_SLOTS=$v timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline > $O/dp_v${v}_r${rep}.json 2> $O/dp_v${v}_r${rep}.err
    echo "slots=$v rep=$rep $(python3 -c "import json; d=json.load(open('$O/dp_v${v}_r${rep}.json')); print(round(d['value'],1), d['dp']['exposed_allreduce_ms'])")"
  done
done
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29599 MMAD_DP_SELFTEST=1 \
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run \
  --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline \
  > $O/prof.log 2>&1
echo prof ok
