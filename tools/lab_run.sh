#!/bin/bash
# Lab: a focused GPU test selection, then bench lines for the given configs.  Usage:
#   bash tools/lab_run.sh TAG "PYTEST -k EXPR or -" "CONFIG [CONFIG...]" [bench args...]
set -u
TAG=$1; KEXPR=$2; CFGS=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$KEXPR" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 50 --warmup 5 "$@" > $OUT/bench_$c.log 2>&1 || { echo "$c failed"; tail -5 $OUT/bench_$c.log; exit 1; }
  grep '^{' $OUT/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], 'enc', d['roofline']['launch_us'], d['roofline']['frac'], 'dec', d['decode_roofline']['launch_us'], d['decode_roofline']['frac'], d['verified'], d['verified_vs_reference_digest'])"
done
echo done
