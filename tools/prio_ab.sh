# frame kernels: wave priority 3 over finish_frame (product, RFEC_WIRE_FRAME_PRIO 2) vs over the header
# bytes and finish_frame (fp4); tools/bin/ab build (tools/build_ab.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prio3
for rep in 1 2 3; do
  for v in fp2 fp4; do
    lib=""; [ $v != fp2 ] && lib="--lib tools/bin/ab/librazor_fec_v1200_$v.so"
    timeout -k 10 300 python tools/wire_bench.py $lib --out gpurun_out/prio3/$v$rep.json > gpurun_out/prio3/$v$rep.log 2>&1 || { tail gpurun_out/prio3/$v$rep.log; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/prio3/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()}, d['verified'])"
  done
done
