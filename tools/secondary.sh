#!/bin/bash
# Secondary configurations (SURVEY §8d parity cases) through bench.py on one GPU:
#   bash tools/secondary.sh <tag>   -> gpurun_out/<tag>/*.json (one bench line each)
set -u
TAG=${1:-sec}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <bench args...>
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
  grep '^{' "$OUT/$name.log" > "$OUT/$name.json"
  python -c "
import json; d=json.load(open('$OUT/$name.json'))
print('  value', d['value'], 'enc', d['roofline']['frac'], 'dec', d.get('decode_roofline', {}).get('frac'), d['config']['workload'])"
}
run c3full --config c3full
run c5 --config c5
run c4_1gpu --config c4
run k16full --k 16 --full-plan --groups 65536
run k24 --k 24 --col 4 --groups 65536
run k12 --k 12 --col 4 --groups 65536
run c3_inplace --in-place
run gpus2_c4 --gpus 2
echo done
