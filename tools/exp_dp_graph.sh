# one-rank RCCL self-test with the all-reduce captured in the graph (bench --graph), vs eager
O=gpurun_out/${1:-dpg}; mkdir -p $O
export PYTHONFAULTHANDLER=1
MMAD_DP_SELFTEST=1 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > $O/dp_graph.json 2> $O/dp_graph.err; rc=$?
echo "graph rc=$rc"; grep -v "UserWarning\|return Variable\|amdgpu.ids" $O/dp_graph.err | tail -15
[ $rc -eq 0 ] || exit $rc
MMAD_DP_SELFTEST=1 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/dp_eager.json 2> $O/dp_eager.err || exit 1
for f in dp_graph dp_eager; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', round(d['value'],1), round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3), d['config']['step_launch'], (d.get('roofline') or {}).get('frac'))"; done
