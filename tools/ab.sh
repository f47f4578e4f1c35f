#!/bin/bash
# Interleaved A/B of two library builds through bench.py on one box (GPU box, repo root):
#   bash tools/ab.sh <tag> <libA> <libB> [rounds] [bench args...]
# libA / libB: librazor_fec.so builds (the product's razor_amd/lib/librazor_fec.so, or an A/B build from
# tools/build_ab.sh).  Each round runs A then B (same args, kernel-own timing); the summary prints the
# value and the encode / decode launch times of every run.  Outputs: gpurun_out/<tag>/{a,b}_<round>.json.
set -u
TAG=$1; A=$2; B=$3; R=${4:-3}; shift 4 2>/dev/null || shift $#
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 "$R"); do
  for side in a b; do
    lib=$A; [ $side = b ] && lib=$B
    timeout -k 10 300 python bench.py --no-cpu --steps 50 --warmup 5 --lib "$lib" "$@" > "$OUT/${side}_$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$side round $r rc=$rc"; tail -5 "$OUT/${side}_$r.log"; exit $rc; fi
    grep '^{' "$OUT/${side}_$r.log" > "$OUT/${side}_$r.json"
    python -c "
import json; d=json.load(open('$OUT/${side}_$r.json'))
print('$side', $r, 'value', d['value'], 'enc_us', d['roofline']['launch_us'], 'frac', d['roofline']['frac'],
      'dec_us', d['decode_roofline']['launch_us'], 'frac', d['decode_roofline']['frac'])"
  done
done
echo done
