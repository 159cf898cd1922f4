set -e -o pipefail
O=gpurun_out/r01k; mkdir -p $O
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline > $O/bench_graph.json 2>$O/bench_graph.err
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --workload fusion --no-cpu-baseline > $O/bench_fusion.json 2>$O/bench_fusion.err
HSA_ENABLE_IPC_MODE_LEGACY=0 MMAD_DP_SELFTEST=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_dp.json 2>$O/bench_dp.err
cat $O/*.json
