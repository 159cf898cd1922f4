#!/bin/bash
# plane-pair lattice tile map A/B (MMAD_ZP_XCD2=0 / 1): equality tests, step kernel times,
# and the PMC traffic of the dominant launch under each map
TAG=${1:-r03zg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return $rc
}
step tests 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_lattice_zp_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_oracle_gpu.py -k "zp or plane or layer4 or config2" || exit 1
for v in 0 1; do
  step fetch_$v 90 env MMAD_ZP_XCD2=$v rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$v -o run --output-format csv -- python3 tools/probe_dominant.py
  step write_$v 90 env MMAD_ZP_XCD2=$v rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$v -o run --output-format csv -- python3 tools/probe_dominant.py
  python3 tools/prof_summary.py traffic $OUT/pmc_fetch_$v $OUT/pmc_write_$v > $OUT/traffic_$v.json 2>&1
  grep -E "hbm_bytes_per_launch|fetch_bytes|write_bytes" $OUT/traffic_$v.json
done
bash tools/gpu_envab.sh ${TAG}ab "lattice_zp" MMAD_ZP_XCD2 0 1
echo session done
