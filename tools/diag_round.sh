timeout -k 10 500 python -u -m pytest tests/test_fusion_configs_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fusion_tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|^E " gpurun_out/fusion_tests.txt | head -30
exit $rc
