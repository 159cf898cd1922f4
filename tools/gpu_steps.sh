#!/bin/bash
# One gpurun call = a list of GPU steps, one per stdin line: "name seconds command ...".
# Each step runs under its own time limit with its output in gpurun_out/<tag>/<name>.log;
# a step ending 0 or 1 (a test failure) lets the next one run, anything else (a fault,
# abort, signal or the time limit) ends the call there.
#   gpurun -- 'bash tools/gpu_steps.sh r04a <<EOF
#   tests 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_x_gpu.py
#   bench 240 python -u bench.py --steps 20 --warmup 5
#   EOF'
# Named drivers: tools/gpu_final.sh (round-end validation), tools/gpu_check.sh (a kernel's
# tests + step trace + bench), tools/gpu_workloads.sh (secondary workloads).
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
while read -r name secs cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue ;; esac
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1 < /dev/null
  rc=$?
  echo "$name rc=$rc"
  tail -4 "$OUT/$name.log" | cut -c1-800
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
echo "session $TAG done"
