#!/bin/bash
# lattice wgrad: layer4 full-size tests, isolated wgrad timings (lattice vs row-gather)
set -o pipefail
OUT=gpurun_out/lat3
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_fullsize_gpu.py -x -q -k "layer4" --timeout 150 > $OUT/t.log 2>&1 || { grep -E "^E|Error" $OUT/t.log | head -20; exit 1; }
tail -1 $OUT/t.log
for M in 1 0; do
  for L in l4c2 l4c1; do
    MMAD_LATTICE=$M timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$M$L -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op wgrad > $OUT/$M$L.log 2>&1 || exit 1
    python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$M$L/run_kernel_stats.csv')):
    if 'wgrad' in r['Name'] or 'lattice' in r['Name']: print('LATTICE=$M $L', r['Name'][:44], round(float(r['AverageNs'])/1e3,1), 'us x', r['Calls'])
"
  done
done
