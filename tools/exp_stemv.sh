#!/bin/bash
# Stem-forward variant timing: rocprof the stem probe under each variant library
#   bash tools/exp_stemv.sh sq_NO_DMA sq_NO_STORE ...   (base = the in-tree library)
set -o pipefail
OUT=gpurun_out/stemv
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for V in base "$@"; do
  if [ $V = base ]; then LP=""; else LP=$PWD/varlib/$V/libmmad_hip.so; fi
  MMAD_LIB_PATH=$LP timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$V -o run --output-format csv -- python3 tools/probe_kernel.py --layer ${LAYER:-stem} --op ${OP:-fwd} --reps 10 > $OUT/p_$V.log 2>&1 || exit 1
  echo "== $V"; python tools/prof_summary.py stats $OUT/p_$V 2 | sed -n 2p
done
