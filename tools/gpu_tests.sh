set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r02b/pytest_gpu.log 2>&1
echo "pytest rc=$?"
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r02b/pytest_gpu.log | tail -30
