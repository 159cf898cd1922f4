# FETCH_SIZE / WRITE_SIZE of the dominant lattice launch under both tile orders
set -o pipefail
O=gpurun_out/${1:-latpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
  MMAD_LAT_MAP=$v timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/f$v -o run --output-format csv -- python3 tools/probe_dominant.py > $O/f$v.log 2>&1 || exit 1
  MMAD_LAT_MAP=$v timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/w$v -o run --output-format csv -- python3 tools/probe_dominant.py > $O/w$v.log 2>&1 || exit 1
  python3 tools/prof_summary.py traffic $O/f$v $O/w$v > $O/traffic$v.json
  echo "MAP=$v"; python3 -c "import json; d=json.load(open('$O/traffic$v.json')); print(d['fetch_bytes_per_launch']/1e6, d['write_bytes_per_launch']/1e6)"
done
