# wire kernels: ping-pong (one datagram ahead) vs three-deep pipeline (two ahead), alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/dab
RFEC_AB_DEPTH3=1 timeout -k 10 300 python -u -m pytest tests/test_wire.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dab/pytest3.log 2>&1 || { tail -20 gpurun_out/dab/pytest3.log; exit 1; }
tail -1 gpurun_out/dab/pytest3.log
for rep in 1 2; do
  timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/dab/a$rep.json > gpurun_out/dab/a$rep.log 2>&1 || exit $?
  RFEC_AB_DEPTH3=1 timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/dab/b$rep.json > gpurun_out/dab/b$rep.log 2>&1 || exit $?
  for v in a b; do python -c "
import json; d=json.load(open('gpurun_out/dab/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()}, d['verified'])"; done
done
