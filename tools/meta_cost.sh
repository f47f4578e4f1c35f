# cost of the encode's header (meta) blocks under rotated sets: default vs DIAGNOSTIC no-meta (256, wrong meta)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mc
for rep in 1 2 3; do
for t in 0 256; do
  timeout -k 10 300 python bench.py --no-cpu --no-verify --tuning $t --steps 60 > gpurun_out/mc/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/mc/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'])"
done; done
