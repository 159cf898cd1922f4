set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/wg
L=l1c,l2c1,l2c2,l3c1,l3c2,l4c1,l4c2
run() { timeout -k 10 120 env "$@" python -u tools/bench_conv.py --no-miopen --layers $L --tag "$* " --reps 20 >> gpurun_out/wg/out.txt 2>&1; }
run X=0
for s in 1 2 3 4 6 8 12; do run MMAD_WGRAD_SPLITS=$s; done
for s in 0 2 3 4 5 6 7 8; do run MMAD_WGRAD_BIG=1 MMAD_WGRAD_SPLITS=$s; done
for s in 0 4 7; do run MMAD_WGRAD_BIG=3 MMAD_WGRAD_SPLITS=$s; done
echo done
