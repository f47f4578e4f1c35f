#!/bin/bash
# Round 6 measurement pass (GPU box, repo root): bash tools/measure_r6.sh <tag>
# pytest -m gpu, smoke, the default bench + its rocprofv3 kernel stats, the receiver-session sweep, the
# session soak, the wire PMC passes.  Every GPU step has its own limit; a crash / fault / timeout stops it.
set -u
TAG=${1:-m}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
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
step rocprof_stats 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py
step rx_4096 300 "${PIN[@]}" python tools/rx_session_bench.py --frames 32768 --batch 4096 --threads 1,8 --reps 3 --out "$OUT/rx_4096.json"
step rx_16384 300 "${PIN[@]}" python tools/rx_session_bench.py --frames 32768 --batch 16384 --threads 8 --modes async --reps 3 --out "$OUT/rx_16384.json"
step soak_rx 400 "${PIN[@]}" python tools/soak_rx.py --seconds ${SOAK_S:-150} --out "$OUT/soak_rx.json"
step pmc_wire 700 bash tools/pmc_wire.sh wire_$TAG
echo done | tee -a "$OUT/steps.log"
