#!/bin/bash
# interleaved single-kernel timing of library variants (HIP events, tools/probe_kernel.py)
#   gpurun -- bash tools/probe_ab.sh "LAYER:OP[:FLAGS] ..." variant1 variant2 ...
#   (variant "base" = the in-tree library; others = variants/NAME/libmmad_hip.so)
CASES=$1; shift
for round in 1 2; do
  for c in $CASES; do
    IFS=: read -r layer op flags <<< "$c"
    for v in "$@"; do
      if [ "$v" = base ]; then lib=""; else lib="variants/$v/libmmad_hip.so"; fi
      MMAD_LIB_PATH=$lib timeout -k 10 120 python3 tools/probe_kernel.py --layer $layer --op $op --reps 20 --time ${flags//,/ } || exit 1
    done
  done
done
