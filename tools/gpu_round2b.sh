# Round-2 closing session: tools/gpu_round.sh (tests, bench, rocprof, PMC traffic) plus the
# secondary workloads (BASELINE configs 3 and 5) and the dominant-dispatch split.
#   gpurun --timeout 1100 -- bash tools/gpu_round2b.sh <tag>
set -e -o pipefail
TAG=${1:-r02z}
bash tools/gpu_round.sh $TAG
OUT=gpurun_out/$TAG
python3 tools/step_breakdown.py $OUT/step.txt > $OUT/breakdown.txt
timeout -k 10 240 python -u bench.py --workload fusion --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $OUT/bench_fusion.json 2>> $OUT/bench.err
timeout -k 10 300 python -u bench.py --workload three --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/bench_three.json 2>> $OUT/bench.err
cat $OUT/bench_fusion.json $OUT/bench_three.json
echo "round2b ok"
