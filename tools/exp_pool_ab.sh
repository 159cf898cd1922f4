set -e -o pipefail
T=${1:-pool4}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
tail -1 gpurun_out/$T/pytest.log
for i in 1 2; do
for L in libmmad_base.so libmmad_hip.so; do
  MMAD_LIB_PATH=$PWD/multimodal_alzheimer_amd/$L timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T/b.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/$T/b.json'));print('$L', 'vol/s', round(d['value'],1), 'ms', round(d['ms_per_step'],3))" | tee -a gpurun_out/$T/bench.txt
done; done
