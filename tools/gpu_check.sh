#!/bin/bash
# GPU-box pass.  Each GPU step has its own time limit; a crash / fault /
# timeout (exit >= 124, 134, 139) stops the script; test failures do not.
# Usage (on the box, from the repo root):
#   bash tools/gpu_check.sh <tag> <mode> [bench args...]
#   mode: full  = smoke + pytest -m gpu + bench + rocprofv3 stats of bench
#         tests = smoke + pytest -m gpu
#         ab    = pytest -m gpu + tools/ab_encode.py
#         bench = bench + rocprofv3 stats
#         pmc   = FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.py)
#         wire  = tools/wire_bench.py + tools/send_bench.py + rocprofv3 stats of the wire bench
#         rx    = receiver + sender tests, tools/send_bench.py, tools/rx_bench.py, tools/e2e_bench.py
#         udp   = UDP tests (CPU + GPU), tools/udp_bench.py (loopback socket -> receiver ingestion)
#         all   = pytest + ab + pmc + bench + rocprofv3 stats
set -u
TAG=${1:-run}; MODE=${2:-full}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a "$OUT/steps.log"
  tail -25 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal exit $rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc
  fi
  return 0
}
case "$MODE" in
  full|tests)
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread ;;
  ab|all)
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread
    step ab 600 python tools/ab_encode.py --out "$OUT/ab.json" ;;
esac
case "$MODE" in
  wire)
    step wire 300 python tools/wire_bench.py --out "$OUT/wire.json"
    step send 300 python tools/send_bench.py --out "$OUT/send.json"
    step wire_rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wprof" -o run -- python tools/wire_bench.py ;;
  rx)
    step pytest_rx 900 python -u -m pytest tests/test_receiver.py tests/test_sender.py -m gpu -q -rs --timeout 120 --timeout-method thread
    step send 300 python tools/send_bench.py --out "$OUT/send.json"
    step rx 600 python tools/rx_bench.py --out "$OUT/rx.json"
    step e2e 300 python tools/e2e_bench.py --out "$OUT/e2e.json" ;;
  udp)
    step pytest_udp 600 python -u -m pytest tests/test_udp.py -q -rs --timeout 120 --timeout-method thread
    step udp 300 python tools/udp_bench.py --out "$OUT/udp.json" ;;
esac
case "$MODE" in
  pmc|all)
    step pmc 900 python tools/pmc_traffic.py --out "$OUT/traffic.json" ;;
esac
case "$MODE" in
  full|bench|all)
    step bench 600 python bench.py "$@"
    step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --no-cpu "$@" ;;
esac
echo done | tee -a "$OUT/steps.log"
