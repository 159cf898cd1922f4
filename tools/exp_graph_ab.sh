# interleaved A/B: eager step vs the captured-graph step (bench.py --graph)
set -o pipefail
O=gpurun_out/${1:-gab}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/eager_$i.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --graph > $O/graph_$i.json 2>> $O/bench.err || exit 1
done
grep -o "\"value\": [0-9.]*" $O/*.json
