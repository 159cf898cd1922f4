#!/bin/bash
# lattice kernel: layer4 full-size tests, then isolated timings (default + variants) and SQ counters
set -o pipefail
OUT=gpurun_out/lat2
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_fullsize_gpu.py -x -q -k "layer4" --timeout 150 > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for V in default nob nomfma; do
  if [ $V = default ]; then LP=""; else LP=varlib/$V/libmmad_hip.so; fi
  for L in l4c2 l4c1; do
    for OP in fwd dgrad; do
    [ $V != default ] && [ $OP = dgrad ] && continue
    MMAD_LIB_PATH=$LP timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$V$L$OP -o run --output-format csv -- python3 tools/probe_kernel.py --layer $L --op $OP > $OUT/$V$L.log 2>&1 || exit 1
    python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$V$L$OP/run_kernel_stats.csv')):
    if 'lattice' in r['Name'] or 'igemm' in r['Name']: print('$V $L $OP', r['Name'][:30], round(float(r['AverageNs'])/1e3,1), 'us x', r['Calls'])
"
    done
  done
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/pmc -o run --output-format csv -- python3 tools/probe_kernel.py --layer l4c2 --op fwd > $OUT/pmc.log 2>&1 || exit 1
python3 - $OUT <<'PY'
import csv, sys, collections
d = sys.argv[1]
k = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/pmc/run_counter_collection.csv")):
    if 'lattice' in r["Kernel_Name"]: k[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(k.items()): print(f"   {c:28s} {sum(v)/len(v):.4g}")
PY
