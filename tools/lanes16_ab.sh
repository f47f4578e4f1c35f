# wire frame kernels: 16-byte lanes (product default) vs 20-byte lanes with LDS transposes
# (build/ab/librazor_fec_v1200_lanes20.so: bash tools/build_ab.sh lanes20 -DRFEC_WIRE_LANES16=0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/l16
for rep in 1 2; do
  timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/l16/a$rep.json > gpurun_out/l16/a$rep.log 2>&1 || { tail gpurun_out/l16/a$rep.log; exit 1; }
  timeout -k 10 300 python tools/wire_bench.py --lib build/ab/librazor_fec_v1200_lanes20.so --out gpurun_out/l16/b$rep.json > gpurun_out/l16/b$rep.log 2>&1 || { tail gpurun_out/l16/b$rep.log; exit 1; }
  for v in a b; do python -c "
import json; d=json.load(open('gpurun_out/l16/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()}, d['verified'])"; done
done
