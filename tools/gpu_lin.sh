#!/bin/bash
# decode block order A/B on one box: step_ab (cold) and alternating bench lines
OUT=gpurun_out/lin; mkdir -p $OUT
timeout -k 10 300 python tools/step_ab.py --cold --rounds 8 --reps 10 --variants default --extra "dec linear=0:16777216;enc linear=16777216:0;both linear=16777216:16777216" --out $OUT/ab.json > $OUT/ab.txt 2>&1; echo ab rc=$?; cat $OUT/ab.txt
for rep in 1 2 3; do
  for tu in 0 16777216; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu --tuning $tu > $OUT/b_${tu}_${rep}.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('$OUT/b_${tu}_${rep}.json'))
print($tu, $rep, d['value'], d['roofline']['launch_us'], d['decode_roofline']['launch_us'], d['verified'])"
  done
done
