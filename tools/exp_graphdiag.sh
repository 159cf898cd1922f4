# graph-mode bench: faulthandler trace of the probe path (default N=1 bench)
O=gpurun_out/${1:-gdiag}; mkdir -p $O
export PYTHONFAULTHANDLER=1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/g_probe.json 2> $O/g_probe.err; rc=$?; echo "probe rc=$rc"
grep -v "UserWarning\|return Variable\|amdgpu.ids" $O/g_probe.err | tail -20
cat $O/g_probe.json
exit $rc
