#!/bin/bash
set -u
mkdir -p gpurun_out/v2
for a in 0 1 2; do timeout -k 10 60 ./tools/bin/svc_vram_probe $a > gpurun_out/v2/vram_$a.json 2>&1; echo "probe $a rc=$?"; done
cat gpurun_out/v2/vram_*.json
SVC_VARIANTS="${SVC_VARIANTS:-svc_w8b}" SVC_ROUNDS=3 bash tools/call_svc.sh
