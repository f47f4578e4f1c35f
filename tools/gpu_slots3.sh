#!/bin/bash
# generic output-mapped decode at k = 24 (6 rows of 4, 2 erasures: 4 of 6 rows idle): slot vs line lanes
set -o pipefail
mkdir -p gpurun_out/slots3
for r in 1 2; do
for t in 0 33554432; do
timeout -k 10 200 python bench.py --k 24 --col 4 --payload 1200 --steps 20 --warmup 5 --no-cpu --tuning $t > gpurun_out/slots3/k24_t${t}_$r.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/slots3/k24_t${t}_$r.log').read().strip().splitlines()[-1])
print('k24 tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], 'dec', d['decode_roofline']['launch_us'], 'verified', d['verified'])
"
done; done
