#!/bin/bash
# full-size layer3/4 tests, then isolated timings of the narrow-tile lattice launches
set -o pipefail
OUT=gpurun_out/latw
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 250 python -u -m pytest tests/test_fullsize_gpu.py -x -q -k "layer3 or layer4" --timeout 150 > $OUT/t.log 2>&1 || { grep -E "^E|Error" $OUT/t.log | head -20; exit 1; }
tail -1 $OUT/t.log
for L in l4c1 l3c1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$L -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op dgrad > $OUT/$L.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$L/run_kernel_stats.csv')):
    if 'lattice' in r['Name'] or 'igemm' in r['Name']: print('$L dgrad', r['Name'][:44], round(float(r['AverageNs'])/1e3,1), 'us x', r['Calls'])
"
done
