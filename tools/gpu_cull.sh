#!/bin/bash
# Tap-culling check (round 5): the culling tests + config 5's in-situ per-conv bar, then a
# same-box A/B of the config-5 bench -- in-tree library (forward + wgrad culling), wgrad
# culling off (MMAD_WGRAD_CULL=0), and the variants/nocull build (-DMMAD_IGEMM_CULL=0) with
# wgrad culling off -- and the config-2 bench (which has no culled tiles) as a control.
#   gpurun -- bash tools/gpu_cull.sh TAG
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_igemm_cull_gpu.py "tests/test_fullsize_oracle_gpu.py::test_full_size_bf16_every_conv_in_situ" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
NOCULL=$GRAFT_REPO_ROOT/variants/nocull/libmmad_hip.so
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload three --steps 6 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/t_cull$i.json 2> $OUT/t_cull$i.err || exit 1
  MMAD_WGRAD_CULL=0 timeout -k 10 300 python -u bench.py --workload three --steps 6 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/t_fwd$i.json 2> $OUT/t_fwd$i.err || exit 1
  MMAD_WGRAD_CULL=0 MMAD_LIB_PATH=$NOCULL timeout -k 10 300 python -u bench.py --workload three --steps 6 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/t_none$i.json 2> $OUT/t_none$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/c2_cull.json 2> $OUT/c2_cull.err || exit 1
MMAD_WGRAD_CULL=0 MMAD_LIB_PATH=$NOCULL timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/c2_none.json 2> $OUT/c2_none.err || exit 1
for f in $OUT/*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value'], 2), round(d['ms_per_step'], 3))"
done
echo session done
