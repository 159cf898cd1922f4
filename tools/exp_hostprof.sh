# host-side profile of the eager step: bench line (host_issue_ms_per_step) + cProfile top
set -o pipefail
O=gpurun_out/${1:-hostprof}; mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/eager.json 2>> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/eager.json')); print(round(d['value'],1), round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3))"
timeout -k 10 300 python -u -m cProfile -o $O/p.out bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/prof_bench.json 2>> $O/bench.err || exit 1
python3 -c "
import pstats; p = pstats.Stats('$O/p.out'); p.sort_stats('tottime').print_stats(45)" > $O/top.txt
head -80 $O/top.txt | tail -55
