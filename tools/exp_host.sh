# host-issue time per step, eager vs graph replay (bench.py host_issue_ms_per_step)
set -o pipefail
O=gpurun_out/${1:-host}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/eager_$i.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --graph > $O/graph_$i.json 2>> $O/bench.err || exit 1
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value'],1), round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3))"; done
nproc; cat /proc/loadavg
