timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -k step -x -q -s --timeout 200 > gpurun_out/diag_cos.txt 2>&1
grep "^cos\|passed\|failed" gpurun_out/diag_cos.txt
