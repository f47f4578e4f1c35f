# k_parse<20>: default registers (78 VGPRs, 1 block / CU) vs waves_per_eu 8 (64 VGPRs + spills, 2 blocks / CU)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pab
RFEC_AB_PARSE8=1 timeout -k 10 300 python -u -m pytest tests/test_wire.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pab/pytest8.log 2>&1 || { tail -20 gpurun_out/pab/pytest8.log; exit 1; }
tail -1 gpurun_out/pab/pytest8.log
for rep in 1 2; do
  timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/pab/a$rep.json > gpurun_out/pab/a$rep.log 2>&1 || exit $?
  RFEC_AB_PARSE8=1 timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/pab/b$rep.json > gpurun_out/pab/b$rep.log 2>&1 || exit $?
  for v in a b; do python -c "
import json; d=json.load(open('gpurun_out/pab/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()})"; done
done
