# store / load policy under rotated buffer sets (cold MALL)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/stune
for rep in 1 2; do
for t in 0 512 64 4 192 2; do
  timeout -k 10 300 python bench.py --no-cpu --sets 2 --tuning $t --steps 60 > gpurun_out/stune/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/stune/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
