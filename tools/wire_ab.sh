#!/bin/bash
# Interleaved A/B of wire-kernel builds through tools/wire_bench.py on one box (GPU box, repo root):
#   bash tools/wire_ab.sh <tag> <rounds> <libA> <libB> [libC ...]
# lib "-": the product build (razor_amd/lib/librazor_fec_v1200.so); others: tools/build_ab.sh outputs.
# Each round runs every build once (kernel-own timing); prints the median time and HBM fraction per kernel.
set -u
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 "$R"); do
  i=0
  for lib in "$@"; do
    i=$((i + 1))
    arg=""; [ "$lib" != "-" ] && arg="--lib $lib"
    timeout -k 10 300 python tools/wire_bench.py $arg --out "$OUT/v${i}_$r.json" > "$OUT/v${i}_$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "build $i ($lib) round $r rc=$rc"; tail -5 "$OUT/v${i}_$r.log"; exit $rc; fi
    python -c "
import json; d=json.load(open('$OUT/v${i}_$r.json'))
print('v$i', $r, ' '.join('%s %.1f %.3f' % (k, x['median_us'], x['frac_of_hbm_peak']) for k, x in d['kernels'].items()), d['verified'])"
  done
done
echo done
