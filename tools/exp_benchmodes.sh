# bench launch modes: default (graph at N=1, probe + cpu baseline), --eager, DP self-test
set -o pipefail
O=gpurun_out/${1:-modes}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graph_step_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || { tail -20 $O/default.err; exit 1; }
timeout -k 10 200 python -u bench.py --eager --no-cpu-baseline > $O/eager.json 2> $O/eager.err || { tail -20 $O/eager.err; exit 1; }
MMAD_DP_SELFTEST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/dp.json 2> $O/dp.err || { tail -20 $O/dp.err; exit 1; }
for f in default eager dp; do python3 -c "
import json; d=json.load(open('$O/$f.json')); r=d.get('roofline') or {}
print('$f', round(d['value'],1), round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3), d['config'].get('step_launch'), r.get('frac'), r.get('probe'), (d.get('cpu_baseline') or {}).get('value'))"; done
