# one-rank RCCL self-test: bucket size vs step time and host enqueue time
set -o pipefail
O=gpurun_out/${1:-dpb}; mkdir -p $O
for i in 1 2; do
for mb in 4 16 64; do
  MMAD_DP_BUCKET_MB=$mb MMAD_DP_SELFTEST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $O/dp_${mb}_$i.json 2>> $O/dp.err || exit 1
  python3 -c "import json; d=json.load(open('$O/dp_${mb}_$i.json')); print($mb, round(d['value'],1), round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3), d['dp'])"
done
done
