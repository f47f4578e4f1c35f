# config 5 encode / decode policies with rotated buffer sets
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c5c
for rep in 1 2; do
for t in 0 512 192 8 8192; do
  timeout -k 10 300 python bench.py --no-cpu --tuning $t --steps 60 --k 32 --payload 256 --col 4 > gpurun_out/c5c/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/c5c/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
