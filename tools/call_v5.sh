#!/bin/bash
set -u
mkdir -p gpurun_out/v5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v5/pt.log 2>&1 || { tail -20 gpurun_out/v5/pt.log; exit 1; }
tail -2 gpurun_out/v5/pt.log
timeout -k 10 300 python bench.py > gpurun_out/v5/bench.json 2> gpurun_out/v5/bench.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/v5/bench2.json 2> gpurun_out/v5/bench2.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v5/prof -o run -- python bench.py > gpurun_out/v5/bench_prof.json 2> gpurun_out/v5/prof.err || exit 1
for f in bench bench2 bench_prof; do python3 -c "
import json,sys; d=json.loads(open('gpurun_out/v5/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('mix_ceiling',{}).get('kernel_vs_ceiling'), d['c4_strong']['value'])"; done
