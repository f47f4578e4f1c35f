#!/bin/bash
# GPU tests, then bench c3 / c5 (kernel-own timing) and rocprofv3 kernel stats of the same commands,
# so the bench's launch_us can be checked against rocprofv3's average per kernel.
set -u
OUT=gpurun_out/${1:-tc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 50 --warmup 5 > $OUT/bench_$c.log 2>&1 || { tail $OUT/bench_$c.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- python bench.py --config $c --no-cpu --steps 50 --warmup 5 > $OUT/rocprof_$c.log 2>&1 || { tail $OUT/rocprof_$c.log; exit 1; }
done
echo done
