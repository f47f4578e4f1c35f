# does a longer warm-up change the steady-state step? (box-to-box variance check)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wu
for rep in 1 2; do
for w in 10 300; do
  timeout -k 10 300 python bench.py --no-cpu --warmup $w --steps 100 > gpurun_out/wu/w$w.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/wu/w$w.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('warmup $w', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'])"
done; done
