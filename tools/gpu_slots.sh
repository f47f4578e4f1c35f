#!/bin/bash
# dense-output row decode: slot lanes (default) vs line lanes, parity tests then alternating bench
set -o pipefail
mkdir -p gpurun_out/slots
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "dense_output or rows or erasure" --timeout 120 --timeout-method thread > gpurun_out/slots/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/slots/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
for t in 0 33554432; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --tuning $t > gpurun_out/slots/t${t}_$r.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/slots/t${t}_$r.log').read().strip().splitlines()[-1])
print('tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], 'dec', d['decode_roofline']['launch_us'], 'verified', d['verified'])
"
done; done
