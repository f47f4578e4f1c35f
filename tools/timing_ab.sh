#!/bin/bash
# bench.py --timing own (kernel-own events, no markers between launches) vs --timing bracket
# (stream events around each call): value, and the roofline launch durations, alternated on one box
set -u
OUT=gpurun_out/${1:-tab}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for t in own bracket; do
    for c in c3 c5; do
      timeout -k 10 300 python bench.py --config $c --no-cpu --timing $t > $OUT/${c}_${t}_$rep.log 2>&1 || { tail $OUT/${c}_${t}_$rep.log; exit 1; }
      python -c "
import json; d=[json.loads(l) for l in open('$OUT/${c}_${t}_$rep.log') if l.startswith('{')][0]
print('$c $t $rep', d['value'], d['ms_per_step'], 'enc', d['roofline']['launch_us'], d['roofline']['frac'], 'dec', d['decode_roofline']['launch_us'], d['decode_roofline']['frac'])"
    done
  done
done
