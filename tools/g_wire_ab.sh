# GPU box: wire tests, then interleaved wire_bench runs of the product build and lab/ builds.  bash tools/g_wire_ab.sh TAG LIB...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wire.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_wire.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python tools/wire_bench.py --reps 10 > $OUT/prod$r.log 2>&1 || exit $?
  for L in "$@"; do timeout -k 10 200 python tools/wire_bench.py --reps 10 --lib $L > $OUT/$(basename $L .so)$r.log 2>&1 || exit $?; done
done
