# drop-in per-call latency: blocking synchronize vs polling the stream
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/di
for rep in 1 2; do
  RFEC_AB_DI_BLOCK=1 timeout -k 10 300 python tools/dropin_bench.py --out gpurun_out/di/block$rep.json > gpurun_out/di/block$rep.log 2>&1 || exit $?
  timeout -k 10 300 python tools/dropin_bench.py --out gpurun_out/di/poll$rep.json > gpurun_out/di/poll$rep.log 2>&1 || exit $?
  for v in block poll; do python -c "
import json; d=json.load(open('gpurun_out/di/$v$rep.json')); print('$v', round(d['generate_gpu_us'],2), round(d['recover_gpu_us'],2), round(d['generate_cpu_us'],2), d['generate_equal'], d['recover_equal'])"; done
done
