#!/bin/bash
# Round-3 session: the new / fixed tests (plane-pair equality incl. the pipelined stage loop,
# MNI ragged geometry, full-size oracle parity, graph modes), the config-2 bench line, the
# pipelined-vs-barrier-first plane-pair A/B (variants/zp_pipe0, built beforehand with
# `python -m multimodal_alzheimer_amd._build --variant zp_pipe0 -DZP_PIPE=0`), PMC traffic
# and SQ counters of the dominant kernel, the MNI bench line.
TAG=${1:-r03d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step tests 420 $PYT -s tests/test_lattice_zp_gpu.py tests/test_mni_geometry_gpu.py tests/test_fullsize_oracle_gpu.py tests/test_graph_step_gpu.py
step bench 200 python -u bench.py --steps 20 --warmup 5
step ab_pipe0 150 env MMAD_LIB_PATH=variants/zp_pipe0/libmmad_hip.so python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/probe_dominant.py
step write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/probe_dominant.py
python3 tools/prof_summary.py traffic $OUT/pmc_fetch $OUT/pmc_write > $OUT/traffic.json
head -8 $OUT/traffic.json
step sqa 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/sqa -o run --output-format csv -- python3 tools/probe_dominant.py
step mni 150 python -u bench.py --size mni --steps 20 --warmup 5
echo session done
