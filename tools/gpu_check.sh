#!/bin/bash
# One GPU-box pass: smoke, the -m gpu suite, a bench line, and a rocprofv3
# kernel-trace summary of the same bench command.  Each GPU step has its own
# time limit; a crash / fault / timeout (exit >= 124) stops the script.
# Usage (on the box, from the repo root): bash tools/gpu_check.sh <tag> [bench args...]
set -u
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal exit $rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc
  fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench 600 python bench.py "$@"
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --no-cpu "$@"
echo done | tee -a "$OUT/steps.log"
