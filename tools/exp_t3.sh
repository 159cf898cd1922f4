set -o pipefail
O=gpurun_out/t3; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for v in 1 0; do
    MMAD_REDUCE_STREAM=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_r${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
grep -o "\"value\": [0-9.]*" $O/bench*.json
