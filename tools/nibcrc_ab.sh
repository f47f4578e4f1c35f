# wire kernels: lane CRC by byte tables (slice-by-16, bank conflicts) vs by nibble tables (2x lookups, conflict-free);
# build/ab2/librazor_fec_v1200_nib.so was rfec_wire.hip with a nibble-table lane CRC (not kept)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/nib
for rep in 1 2; do
  timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/nib/a$rep.json > gpurun_out/nib/a$rep.log 2>&1 || { tail gpurun_out/nib/a$rep.log; exit 1; }
  timeout -k 10 300 python tools/wire_bench.py --lib build/ab2/librazor_fec_v1200_nib.so --out gpurun_out/nib/b$rep.json > gpurun_out/nib/b$rep.log 2>&1 || { tail gpurun_out/nib/b$rep.log; exit 1; }
  for v in a b; do python -c "
import json; d=json.load(open('gpurun_out/nib/$v$rep.json')); print('$v', {k:x['median_us'] for k,x in d['kernels'].items()}, d['verified'])"; done
done
