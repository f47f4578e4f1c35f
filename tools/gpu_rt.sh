#!/bin/bash
# run-time-k row encode: parity tests, then k = 12 / 24 (col 4) and k = 20 (col 5) against the plan-driven kernel
set -o pipefail
mkdir -p gpurun_out/rt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_plan_encode or sender or rows_fixture or dense_output" --timeout 120 --timeout-method thread > gpurun_out/rt/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/rt/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "--k 20 --col 5" "--k 32 --col 8" "--k 48 --col 16"; do
for t in 0 1; do
timeout -k 10 200 python bench.py $cfg --payload 1200 --steps 20 --warmup 5 --no-cpu --tuning $t > gpurun_out/rt/run.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/rt/run.log').read().strip().splitlines()[-1])
print('$cfg tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], d['roofline']['frac'], 'dec', d['decode_roofline']['launch_us'], d['decode_roofline']['frac'], 'verified', d['verified'])
"
done; done
