#!/bin/bash
# Round 6 quick pass (GPU box, repo root): bash tools/r6_quick.sh <tag>
# pytest -m gpu, smoke, the default bench, the receiver-session bench (thread sweep).
set -u
TAG=${1:-q}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a "$OUT/steps.log"
  tail -4 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal exit $rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc
  fi
  return 0
}
LOCAL=$(bash tools/gpu_local_cpus.sh)
PIN=(); [ -n "$LOCAL" ] && PIN=(taskset -c "$LOCAL")
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
step rx_session 400 "${PIN[@]}" python tools/rx_session_bench.py --frames 32768 --threads ${RX_THREADS:-1,4,8,16} --reps 3 --out "$OUT/rx_session.json"
echo done | tee -a "$OUT/steps.log"
