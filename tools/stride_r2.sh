#!/bin/bash
# Slot stride A/B with the round-2 kernels (output-mapped encode, dense decode):
# packed 1,200 B vs 64-B aligned 1,216 B vs line-aligned 1,280 B, alternated
mkdir -p gpurun_out/stride_r2
for rep in 1 2; do
  for st in 1200 1216 1280; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu --stride $st > gpurun_out/stride_r2/b_${st}_${rep}.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/stride_r2/b_${st}_${rep}.json'))
print($st, $rep, d['value'], d['roofline']['launch_us'], d['decode_roofline']['launch_us'], d['verified'])"
  done
done
