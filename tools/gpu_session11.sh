#!/bin/bash
# SQ counters of the dominant kernel (plane-pair lattice, layer4.0.conv2 forward), one pass
# per counter group (tools/probe_dominant.py)
TAG=${1:-r03q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step sqa 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS -d $OUT/sqa -o run --output-format csv -- python3 tools/probe_dominant.py
step sqb 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/sqb -o run --output-format csv -- python3 tools/probe_dominant.py
step sqc 90 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT GRBM_COUNT -d $OUT/sqc -o run --output-format csv -- python3 tools/probe_dominant.py
python3 - <<'PY'
import csv, collections, glob, os
out = os.environ.get("OUT_DIR", "")
PY
for d in sqa sqb sqc; do
  python3 -c "
import csv, collections, sys
rows = list(csv.DictReader(open('$OUT/$d/run_counter_collection.csv')))
acc = collections.defaultdict(list)
for r in rows:
    if 'lattice_zp_kernel' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(acc.items()):
    v = sorted(v); print('$d', k, 'n=%d median=%.4g' % (len(v), v[len(v)//2]))
" | tee -a $OUT/counters.txt
done
echo session done
