#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "conv3d_fwd_bwd" -x -q --timeout 120 --timeout-method thread > gpurun_out/kt.log 2>&1; tail -2 gpurun_out/kt.log
for P in 0 1; do
  MMAD_SETPRIO=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prio/p_$P -o run --output-format csv -- python3 tools/probe_kernel.py --layer l4c2 --op fwd --reps 20 > gpurun_out/prio_$P.log 2>&1 || exit 1
  python tools/prof_summary.py stats gpurun_out/prio/p_$P 2 | sed -n 2p
done
bash tools/exp_ab.sh MMAD_SETPRIO 0 1 3
