#!/bin/bash
# generic output-mapped decode: slot lanes (default) vs line lanes; parity tests first
set -o pipefail
mkdir -p gpurun_out/slots2
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "dense_output or erasure or rows" --timeout 120 --timeout-method thread > gpurun_out/slots2/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/slots2/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for t in 0 33554432; do
timeout -k 10 200 python bench.py --k 12 --col 4 --payload 1200 --steps 20 --warmup 5 --no-cpu --tuning $t > gpurun_out/slots2/k12_t${t}_$r.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/slots2/k12_t${t}_$r.log').read().strip().splitlines()[-1])
print('k12 tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], 'dec', d['decode_roofline']['launch_us'], d['decode_roofline']['kernels'][:40], 'verified', d['verified'])
"
done; done
