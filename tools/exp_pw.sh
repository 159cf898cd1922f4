#!/bin/bash
# Patch wgrad (layer1) check: full-size layer1 test, isolated wgrad time both ways, step table.
set -o pipefail
OUT=gpurun_out/pw
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -k "layer1" -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for P in 0 1; do
  MMAD_PWGRAD=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$P -o run --output-format csv -- python3 tools/probe_kernel.py --layer l1c --op wgrad --reps 10 > $OUT/p_$P.log 2>&1 || exit 1
  python tools/prof_summary.py stats $OUT/p_$P 3 | sed -n 2,3p
done
bash tools/prof_step.sh step_g
