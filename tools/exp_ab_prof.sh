# A/B of one env switch: tests under B, interleaved bench, rocprof step table per value
#   bash tools/exp_ab_prof.sh <tag> <VAR> <A> <B> "<pytest args>" "<kernel regex>"
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
env "$2=$4" timeout -k 10 400 python -u -m pytest $5 -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in "$3" "$4"; do
    env "$2=$v" timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
grep -o "\"value\": [0-9.]*" $O/bench*.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$3" "$4"; do
  env "$2=$v" timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_$v.log 2>&1 || exit 1
  python3 tools/prof_summary.py step $O/prof_$v > $O/step_$v.txt
  echo "== $2=$v"; grep -E "$6" $O/step_$v.txt; tail -1 $O/step_$v.txt
done
