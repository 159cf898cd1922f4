#!/bin/bash
# Round-3 second session: the fixed / new tests (plane-pair equality, full-size bf16 bounds,
# MNI ragged geometry), PMC traffic + SQ counters of the dominant kernel, bench lines
# (config 2, MNI, configs 3 and 5).  Same step rules as gpu_session.sh.
TAG=${1:-r03b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step tests 400 $PYT -s tests/test_lattice_zp_gpu.py tests/test_mni_geometry_gpu.py tests/test_fullsize_oracle_gpu.py
step fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/probe_dominant.py
step write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/probe_dominant.py
python3 tools/prof_summary.py traffic $OUT/pmc_fetch $OUT/pmc_write > $OUT/traffic.json
cat $OUT/traffic.json | head -8
step sqa 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/sqa -o run --output-format csv -- python3 tools/probe_dominant.py
step sqb 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/sqb -o run --output-format csv -- python3 tools/probe_dominant.py
step bench 240 python -u bench.py --steps 20 --warmup 5
step mni 240 python -u bench.py --size mni --steps 20 --warmup 5
step mni0 240 env MMAD_LATTICE_RAGGED=0 python -u bench.py --size mni --steps 20 --warmup 5
step fusion 240 python -u bench.py --workload fusion --steps 10 --warmup 3
step three 300 python -u bench.py --workload three --steps 5 --warmup 2
echo session done
