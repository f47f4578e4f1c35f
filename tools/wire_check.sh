#!/bin/bash
# wire GPU tests, the wire bench (kernel-own timing) twice, rocprofv3 kernel stats of the wire bench
set -u
OUT=gpurun_out/${1:-wc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wire.py tests/test_receiver.py tests/test_sender.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 300 python tools/wire_bench.py --out $OUT/wire$r.json > $OUT/wire$r.log 2>&1 || { tail $OUT/wire$r.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/wire$r.json')); print({k:(x['median_us'],x['frac_of_hbm_peak']) for k,x in d['kernels'].items()}, d['verified'], d['timing'][:20])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/wire_bench.py --reps 20 > $OUT/rocprof.log 2>&1 || { tail $OUT/rocprof.log; exit 1; }
echo done
