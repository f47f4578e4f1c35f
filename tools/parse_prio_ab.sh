# parse: wave priority 3 over the payload store (pp1), the batch header pass (pp3), both (pp4) vs none
# (product, pp0); tools/bin/ab builds (tools/build_ab.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pprio2
for rep in 1 2 3; do
  for v in pp0 pp1 pp3 pp4; do
    lib=""; [ $v != pp0 ] && lib="--lib tools/bin/ab/librazor_fec_v1200_$v.so"
    timeout -k 10 300 python tools/wire_bench.py $lib --out gpurun_out/pprio2/$v$rep.json > gpurun_out/pprio2/$v$rep.log 2>&1 || { tail gpurun_out/pprio2/$v$rep.log; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/pprio2/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()}, d['verified'])"
  done
done
