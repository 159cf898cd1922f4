#!/bin/bash
# generic env A/B: kernel tests once, then bench_conv + bench.py with each env setting
#   exp_ab.sh TAG "ENV=a" "ENV=b" ...
set -e -o pipefail
T=$1; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 60 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
tail -1 gpurun_out/$T/pytest.log
for e in "$@"; do
  env $e timeout -k 10 120 python -u tools/bench_conv.py --no-miopen --tag "$e " >> gpurun_out/$T/conv.txt 2>&1
  env $e timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T/b.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/$T/b.json'));print('$e', 'vol/s', round(d['value'],1), 'ms', round(d['ms_per_step'],3))" >> gpurun_out/$T/bench.txt
done
grep -v amdgpu.ids gpurun_out/$T/conv.txt; cat gpurun_out/$T/bench.txt
