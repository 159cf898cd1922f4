#!/bin/bash
# A/B of library variants built by `python -m multimodal_alzheimer_amd._build --variant NAME -D...`
#   gpurun -- bash tools/ab_variants.sh TAG NAME1 NAME2 ...   (base = the in-tree library)
set -e
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/$TAG/base_$i.json 2> gpurun_out/$TAG/base_$i.err
  for v in "$@"; do
    MMAD_LIB_PATH=variants/$v/libmmad_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/$TAG/${v}_$i.json 2> gpurun_out/$TAG/${v}_$i.err
  done
done
for f in gpurun_out/$TAG/*.json; do
  python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value'], 2), round(d['ms_per_step'], 4))"
done
