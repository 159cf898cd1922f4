#!/bin/bash
# Stem-forward check: stem parity tests, then bench A/B (MMAD_STEM_QUAD=0/1) and the kernel
# time of both forms from a rocprof pass over the stem probe.
set -o pipefail
OUT=gpurun_out/stem
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py tests/test_kernels_gpu.py -k "stem or config2" -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/tests.log | head -30
[ $rc -ne 0 ] && exit $rc
for Q in 0 1; do
  MMAD_STEM_QUAD=$Q timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof$Q -o run --output-format csv -- python3 tools/probe_kernel.py --layer stem --op fwd --reps 10 > $OUT/prof$Q.log 2>&1 || exit 1
  python tools/prof_summary.py stats $OUT/prof$Q 6 | tee $OUT/stats$Q.txt | head -8
done
bash tools/exp_ab.sh MMAD_STEM_QUAD 0 1 2
