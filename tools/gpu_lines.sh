#!/bin/bash
# output-mapped encode for plans with short lines (the sender's full plans) vs the matrix kernel (RFEC_TUNE_FLAT_ENCODE)
set -o pipefail
mkdir -p gpurun_out/lines
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_flex_dropin.py tests/test_dropin.py -m gpu -x -q -k "sender or full_plan or cascade or row_plan or flex" --timeout 120 --timeout-method thread > gpurun_out/lines/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/lines/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for t in 0 65536; do
timeout -k 10 200 python bench.py --full-plan --steps 20 --warmup 5 --no-cpu --tuning $t > gpurun_out/lines/run.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/lines/run.log').read().strip().splitlines()[-1])
print('full tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], d['roofline']['frac'], d['roofline']['traffic'], 'dec', d['decode_roofline']['launch_us'], 'verified', d['verified'])
"
done; done
