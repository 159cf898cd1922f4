set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ew
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ew/new -o run --output-format csv -- python3 tools/bench_ew.py > gpurun_out/ew/new.log 2>&1
MMAD_POOL_ROWS=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ew/old -o run --output-format csv -- python3 tools/bench_ew.py > gpurun_out/ew/old.log 2>&1
python tools/prof_summary.py stats gpurun_out/ew/new 14
python tools/prof_summary.py stats gpurun_out/ew/old 14
