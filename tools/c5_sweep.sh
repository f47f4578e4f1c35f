# config 5 (k = 32, 8 rows of 4, S = 256) decode variants
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c5s
for rep in 1 2; do
for t in 0 8 8192 4096; do
  timeout -k 10 300 python bench.py --no-cpu --tuning $t --steps 50 --k 32 --payload 256 --col 4 > gpurun_out/c5s/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/c5s/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us'], d['decode_roofline']['launch_us'], d['decode_roofline']['frac'], d['verified'])"
done; done
