#!/bin/bash
set -u
mkdir -p gpurun_out/e2e
LOCAL=$(bash tools/gpu_local_cpus.sh)
echo "local cpus: $LOCAL"
timeout -k 10 300 python tools/e2e_step.py > gpurun_out/e2e/unpinned.json 2>/dev/null || exit 1
timeout -k 10 300 taskset -c "$LOCAL" python tools/e2e_step.py > gpurun_out/e2e/pinned.json 2>/dev/null || exit 1
timeout -k 10 200 taskset -c "$LOCAL" python tools/h2d_probe.py > gpurun_out/e2e/h2d_pinned.json 2>/dev/null || exit 1
for f in unpinned pinned; do python3 -c "
import json
for line in open('gpurun_out/e2e/$f.json'):
    d=json.loads(line); print('$f', d['workload'][:6], d['encode_e2e_gibps'], d['decode_e2e_gibps'], d['step_e2e_gibps'], 'h2d', d['encode_us']['h2d_us'], d['decode_us']['h2d_us'], 'gather', d['encode_us']['gather_us'], d['decode_us']['gather_us'])"; done
cat gpurun_out/e2e/h2d_pinned.json
