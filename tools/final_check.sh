#!/bin/bash
# The driver's round-end order on one box: pytest -m gpu, smoke, default bench (CPU baseline included),
# then rocprofv3 kernel stats of the default bench command.
set -u
OUT=gpurun_out/${1:-fin}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu > $OUT/rocprof.log 2>&1 || { tail $OUT/rocprof.log; exit 1; }
echo done
