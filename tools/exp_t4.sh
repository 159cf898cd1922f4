# full -m gpu suite, bench A/B of the twin switch, rocprof step table (round-2 experiments)
set -o pipefail
O=gpurun_out/${1:-t4}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for v in 1 0; do
    MMAD_TWIN=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_t${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
grep -o "\"value\": [0-9.]*" $O/bench*.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1 || exit 1
python3 tools/prof_summary.py step $O/prof > $O/step.txt && python3 tools/step_breakdown.py $O/step.txt > $O/breakdown.txt
tail -1 $O/step.txt; cat $O/breakdown.txt
