#!/bin/bash
# c5 dense decode: flat lanes (default) vs output-mapped slot lanes (RFEC_TUNE_OUT_DECODE), alternating
set -o pipefail
mkdir -p gpurun_out/c5slots
for r in 1 2 3; do
for t in 0 2097152; do
timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu --tuning $t > gpurun_out/c5slots/t${t}_$r.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/c5slots/t${t}_$r.log').read().strip().splitlines()[-1])
print('tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], 'dec', d['decode_roofline']['launch_us'], 'verified', d['verified'])
"
done; done
