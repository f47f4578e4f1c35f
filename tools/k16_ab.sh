# k = 16 full plan (4x4, 8 lines): one-launch cascade decode (default) vs peel + replay (4096), rotated sets
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k16
for rep in 1 2; do
for t in 0 4096; do
  timeout -k 10 300 python bench.py --no-cpu --full-plan --k 16 --tuning $t --steps 40 > gpurun_out/k16/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/k16/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
