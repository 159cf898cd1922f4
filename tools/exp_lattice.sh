#!/bin/bash
# Lattice-conv check: full-size layer tests, then bench A/B (MMAD_LATTICE=0/1), kernel stats.
set -o pipefail
OUT=gpurun_out/lat
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/full.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/full.log | head -30
[ $rc -ne 0 ] && exit $rc
for L in 0 1 0 1; do
  MMAD_LATTICE=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$L.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_$L.json'));print('LATTICE=$L', round(d['value'],1), round(d['ms_per_step'],3))"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $OUT/prof.log 2>&1 || exit 1
python tools/prof_summary.py stats $OUT/prof 25 > $OUT/stats.txt; head -28 $OUT/stats.txt
