#!/bin/bash
# Interleaved runs of several library builds through bench.py on one box (GPU box, repo root):
#   bash tools/abn.sh <tag> <rounds> <lib>... -- [bench args...]
# lib: a librazor_fec.so build path, or `-` for the product build.  Each round runs every lib in turn
# (kernel-own timing).  Outputs gpurun_out/<tag>/<i>_<round>.json and one summary line per run.
set -u
TAG=$1; R=$2; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ $# -gt 0 ] && shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 "$R"); do
  for i in "${!LIBS[@]}"; do
    lib=${LIBS[$i]}; la=(); [ "$lib" != "-" ] && la=(--lib "$lib")
    timeout -k 10 300 python bench.py --no-cpu --steps 50 --warmup 5 "${la[@]}" "$@" > "$OUT/${i}_$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "lib $i round $r rc=$rc"; tail -5 "$OUT/${i}_$r.log"; exit $rc; fi
    grep '^{' "$OUT/${i}_$r.log" > "$OUT/${i}_$r.json"
    python -c "
import json; d=json.load(open('$OUT/${i}_$r.json'))
print('$i', '$(basename "$lib")', $r, 'value', d['value'], 'enc_us', d['roofline']['launch_us'], 'frac', d['roofline']['frac'],
      'dec_us', d['decode_roofline']['launch_us'], 'frac', d['decode_roofline']['frac'])"
  done
done
echo done
