#!/bin/bash
# Stem weight-gradient check: stem parity tests, then the wgrad kernel time of both forms.
set -o pipefail
OUT=gpurun_out/stemw
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -k "stem" -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/tests.log | head -30
[ $rc -ne 0 ] && exit $rc
for Q in 0 1; do
  MMAD_STEM_WG2=$Q timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof$Q -o run --output-format csv -- python3 tools/probe_kernel.py --layer stem --op wgrad --reps 10 > $OUT/prof$Q.log 2>&1 || exit 1
  python tools/prof_summary.py stats $OUT/prof$Q 4 | sed -n 2,4p
done
