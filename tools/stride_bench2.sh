# bench.py at the packed 1200-B stride vs 1216 / 1280, alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sb2
for rep in 1 2 3; do
for st in 0 1216 1280; do
  timeout -k 10 300 python bench.py --no-cpu --stride $st --steps 100 > gpurun_out/sb2/s$st.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/sb2/s$st.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('stride $st', d['value'], d['roofline']['launch_us'], d['decode_roofline']['launch_us'], d['verified'])"
done; done
