#!/bin/bash
# lattice8 (layer3): full-size tests, isolated fwd / dgrad timings vs the row-gather GEMM
set -o pipefail
OUT=gpurun_out/lat8
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_fullsize_gpu.py -x -q -k "layer3" --timeout 150 > $OUT/t.log 2>&1 || { grep -E "^E|Error" $OUT/t.log | head -20; exit 1; }
tail -1 $OUT/t.log
for M in 1 0; do
  for L in l3c2 l3c1; do
    for OP in fwd dgrad; do
      MMAD_LATTICE8=$M timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$M$L$OP -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP > $OUT/$M$L$OP.log 2>&1 || exit 1
      python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$M$L$OP/run_kernel_stats.csv')):
    if 'lattice' in r['Name'] or 'igemm' in r['Name']: print('L8=$M $L $OP', r['Name'][:36], round(float(r['AverageNs'])/1e3,1), 'us x', r['Calls'])
"
    done
  done
done
