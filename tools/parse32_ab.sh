# k_parse<32> (datagram slots > 1,280 B, e.g. 1,504-B receive slots): default registers vs 64 (two blocks / CU)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p32
RFEC_AB_PARSE32_8=1 timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_udp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p32/pytest8.log 2>&1 || { tail -20 gpurun_out/p32/pytest8.log; exit 1; }
tail -1 gpurun_out/p32/pytest8.log
for rep in 1 2; do
  timeout -k 10 300 python tools/wire_bench.py --dstride 1504 --out gpurun_out/p32/a$rep.json > gpurun_out/p32/a$rep.log 2>&1 || exit $?
  RFEC_AB_PARSE32_8=1 timeout -k 10 300 python tools/wire_bench.py --dstride 1504 --out gpurun_out/p32/b$rep.json > gpurun_out/p32/b$rep.log 2>&1 || exit $?
  for v in a b; do python -c "
import json; d=json.load(open('gpurun_out/p32/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()}, d['verified'])"; done
done
