# decode / encode vs slot stride (rotated sets): is the decode's gain at 1216 the 64-B alignment?
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ss
for rep in 1 2; do
for st in 1200 1216 1232 1248 1280; do
  timeout -k 10 300 python bench.py --no-cpu --stride $st --steps 60 > gpurun_out/ss/s$st.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/ss/s$st.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('stride $st', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
