# session push cost, old vs new host code: build/ab/librazor_fec_v1200_old.so is the previous rfec_host.c
# linked against the current kernel objects (see DESIGN.md section 8 for how it was made and the result)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sab
for rep in 1 2; do
timeout -k 10 300 python tools/session_bench.py --lib build/ab/librazor_fec_v1200_old.so --out gpurun_out/sab/old$rep.json > gpurun_out/sab/old$rep.log 2>&1 || { tail gpurun_out/sab/old$rep.log; exit 1; }
timeout -k 10 300 python tools/session_bench.py --out gpurun_out/sab/new$rep.json > gpurun_out/sab/new$rep.log 2>&1 || { tail gpurun_out/sab/new$rep.log; exit 1; }
for v in old new; do python -c "
import json; d=json.load(open('gpurun_out/sab/$v$rep.json'))
print('$v', {b:(round(x['us_per_push'],1), round(x['host_us_per_push'],1), round(x['kernel_us_per_push'],1), round(x['d2h_us_per_push'],1), x['recovered']) for b,x in d['batches'].items()})"; done
done
