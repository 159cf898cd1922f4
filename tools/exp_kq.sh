# quick check of a kernel change: named test files, then bench + rocprof stats of the step
#   bash tools/exp_kq.sh <tag> "<pytest paths>" "<kernel-name regex>"
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest $2 -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench.json 2>> $O/bench.err || exit 1
grep -o "\"value\": [0-9.]*" $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1 || exit 1
python3 tools/prof_summary.py step $O/prof > $O/step.txt
grep -E "$3" $O/step.txt; tail -1 $O/step.txt
