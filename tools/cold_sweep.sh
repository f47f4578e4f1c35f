# encode / decode mapping variants with rotated buffer sets (cold MALL)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cold
for rep in 1 2; do
for t in 0 8192 8 24576; do
  timeout -k 10 300 python bench.py --no-cpu --sets 2 --tuning $t --steps 60 $EXTRA > gpurun_out/cold/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/cold/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
for st in 1216 1280; do
  timeout -k 10 300 python bench.py --no-cpu --sets 2 --stride $st --steps 60 > gpurun_out/cold/s$st.log 2>&1 || exit $?
  grep '^{' gpurun_out/cold/s$st.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('stride $st', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done
