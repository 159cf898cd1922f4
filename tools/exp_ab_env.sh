# interleaved A/B of one env switch on the bench (round-2 experiments):
#   bash tools/exp_ab_env.sh <tag> <VAR> <valueA> <valueB> [reps]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for i in $(seq 1 ${5:-3}); do
  for v in "$3" "$4"; do
    env "$2=$v" timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_${v}_$i.json 2>> $O/bench.err || exit 1
  done
done
grep -o "\"value\": [0-9.]*" $O/bench*.json
