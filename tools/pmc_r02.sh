#!/bin/bash
# SQ counter passes (two --pmc runs each) over the round-2 kernels, summarised into
# gpurun_out/pmc_r02.txt:  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_r02.txt
: > $OUT
for spec in "l4c2 fwd lattice_conv_kernel" "l4c2 wgrad lattice_wgrad" "stem fwd stem_fwdq" "stem wgrad stem_wgrad2" "l1c wgrad pwgrad" "l1c fwd patch_conv" "l3c2 fwd lattice8"; do
  set -- $spec
  echo "== $1 $2 ($3)" >> $OUT
  bash tools/pmc_kernel.sh $1 $2 $3 > gpurun_out/pmc_tmp.txt 2>&1 || exit 1
  cat gpurun_out/pmc_tmp.txt >> $OUT
  python3 - gpurun_out/pmc_tmp.txt >> $OUT <<'PY'
import sys
v = {}
for line in open(sys.argv[1]):
    p = line.split()
    if len(p) == 2:
        try: v[p[0]] = float(p[1])
        except ValueError: pass
if "GRBM_GUI_ACTIVE" in v and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
    cyc = v["GRBM_GUI_ACTIVE"] / 8
    print(f"   -> kernel cycles {cyc:.4g}; MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}")
PY
done
cat $OUT
