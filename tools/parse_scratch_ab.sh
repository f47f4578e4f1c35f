# parse: header array kept out of scratch (byte_at select chain behind an empty asm, product) vs the
# round-2 m7 build (build/ab/librazor_fec_v1200_lanes20.so, same parse source before the change)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ps
for rep in 1 2 3; do
  timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/ps/a$rep.json > gpurun_out/ps/a$rep.log 2>&1 || { tail gpurun_out/ps/a$rep.log; exit 1; }
  timeout -k 10 300 python tools/wire_bench.py --lib build/ab/librazor_fec_v1200_lanes20.so --out gpurun_out/ps/b$rep.json > gpurun_out/ps/b$rep.log 2>&1 || { tail gpurun_out/ps/b$rep.log; exit 1; }
  for v in a b; do python -c "
import json; d=json.load(open('gpurun_out/ps/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()}, d['verified'])"; done
done
