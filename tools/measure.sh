#!/bin/bash
# The round's standard GPU measurement pass (GPU box, repo root):
#   bash tools/measure.sh <tag>
# pytest -m gpu, smoke, drop-in group bench, the default bench (the driver's command) and the
# rocprofv3 kernel stats of that same command, c3full / c5 lines + stats, the r:w mix probe, the
# end-to-end step, wire bench + stats, PMC traffic passes (FETCH_SIZE / WRITE_SIZE) for c3, c5, c3full and c5's packed-record decode.  Every GPU step has its own limit; a crash /
# fault / timeout stops the script.
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
  tail -4 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal exit $rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc
  fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
LOCAL=$(bash tools/gpu_local_cpus.sh)  # the drop-in bench pinned to the GPU's NUMA node
if [ -n "$LOCAL" ]; then step group_bench 200 taskset -c "$LOCAL" ./razor_amd/lib/fec_dropin_group_bench 2000
else step group_bench 200 ./razor_amd/lib/fec_dropin_group_bench 2000; fi
step bench 400 python bench.py
step rocprof_stats 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py
step bench_c3full 400 python bench.py --config c3full --no-cpu
step bench_c5 400 python bench.py --config c5 --no-cpu
step rocprof_stats_c3full 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3full" -o run -- python bench.py --config c3full --no-cpu --steps 20 --warmup 5
step rocprof_stats_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run -- python bench.py --config c5 --no-cpu --steps 20 --warmup 5
step mix 200 python tools/mix_probe.py
if [ -n "$LOCAL" ]; then step e2e 400 taskset -c "$LOCAL" python tools/e2e_step.py --mem both
else step e2e 400 python tools/e2e_step.py --mem both; fi
step wire_bench 300 python tools/wire_bench.py --out "$OUT/wire.json"
step rocprof_wire 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_wire" -o run -- python tools/wire_bench.py --reps 5
step pmc_c3 600 python tools/pmc_traffic.py --out "$OUT/traffic_c3.json" -- --steps 10 --warmup 2 --c4-steps 0 --sub-steps 0
step pmc_c5 600 python tools/pmc_traffic.py --out "$OUT/traffic_c5.json" -- --config c5 --steps 10 --warmup 2
step pmc_c3full 600 python tools/pmc_traffic.py --out "$OUT/traffic_c3full.json" -- --config c3full --steps 10 --warmup 2
step pmc_c5p 600 python tools/pmc_traffic.py --out "$OUT/traffic_c5p.json" -- --config c5 --packed-decode --steps 10 --warmup 2
echo done | tee -a "$OUT/steps.log"
