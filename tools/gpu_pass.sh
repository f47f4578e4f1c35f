#!/bin/bash
# The standard GPU pass, in the driver's round-end order: pytest -m gpu, smoke, the default bench
# (CPU baseline included), rocprofv3 kernel stats of the same bench command.  Usage: tools/gpu_pass.sh NAME [STEPS]
#   STEPS: any of tests,smoke,bench,prof (default: all four).  Outputs under gpurun_out/NAME/.
set -u
OUT=gpurun_out/${1:-pass}; STEPS=${2:-tests,smoke,bench,prof}; mkdir -p $OUT; export TMPDIR=/tmp
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=15 \
    > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
if has smoke; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
if has bench; then
  timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
  grep '^{' $OUT/bench.log
fi
if has prof; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu \
    > $OUT/rocprof.log 2>&1 || { tail $OUT/rocprof.log; exit 1; }
  cat $OUT/prof/run_kernel_stats.csv | cut -d, -f1-4 | head -8
fi
echo done
