#!/bin/bash
# run-time-k row decode: parity tests, then strip-mode row layouts against the plan-driven decode (RFEC_TUNE_GENERIC)
set -o pipefail
mkdir -p gpurun_out/rtdec
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "dense_output or header_rejections or row_plan_encode" --timeout 120 --timeout-method thread > gpurun_out/rtdec/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/rtdec/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "--k 24 --col 4" "--k 20 --col 3" "--k 12 --col 4"; do
for t in 0 33554432; do
timeout -k 10 200 python bench.py $cfg --payload 1200 --steps 20 --warmup 5 --no-cpu --tuning $t > gpurun_out/rtdec/run.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/rtdec/run.log').read().strip().splitlines()[-1])
print('$cfg tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], d['roofline']['frac'], 'dec', d['decode_roofline']['launch_us'], d['decode_roofline']['frac'], 'verified', d['verified'])
"
done; done
