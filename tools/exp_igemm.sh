#!/bin/bash
# igemm tile-configuration A/B: bit-exactness vs the default and per-conv timing per config
set -e -o pipefail
T=${1:-ig}; shift || true
CFGS=${*:-5 6}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$T
timeout -k 10 60 python -u tools/exp_igemm.py gpurun_out/$T/base.pt > gpurun_out/$T/cmp.txt 2>&1
for c in $CFGS; do
  MMAD_IGEMM_BIG=$c timeout -k 10 60 python -u tools/exp_igemm.py gpurun_out/$T/c$c.pt >> gpurun_out/$T/cmp.txt 2>&1
  timeout -k 10 60 python -u tools/exp_igemm.py --cmp gpurun_out/$T/base.pt gpurun_out/$T/c$c.pt >> gpurun_out/$T/cmp.txt 2>&1
done
timeout -k 10 90 python -u tools/bench_conv.py --no-miopen --layers l3c1,l3c2,l4c1,l4c2 --tag base: > gpurun_out/$T/conv.txt 2>&1
for c in $CFGS; do
  MMAD_IGEMM_BIG=$c timeout -k 10 90 python -u tools/bench_conv.py --no-miopen --layers l3c1,l3c2,l4c1,l4c2 --tag c$c: >> gpurun_out/$T/conv.txt 2>&1
done
rm -f gpurun_out/$T/*.pt
cat gpurun_out/$T/cmp.txt gpurun_out/$T/conv.txt
