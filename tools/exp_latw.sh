#!/bin/bash
# Lattice wgrad check: full-size layer tests, then isolated wgrad times and the step table.
set -o pipefail
OUT=gpurun_out/latw
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -k "layer4 or layer3" -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for L in l4c2 l4c1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$L -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op wgrad --reps 10 > $OUT/p_$L.log 2>&1 || exit 1
  python tools/prof_summary.py stats $OUT/p_$L 3 | sed -n 2,3p
done
bash tools/prof_step.sh step_d
