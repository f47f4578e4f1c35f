#!/bin/bash
# Lab: focused GPU tests, one bench config, rocprofv3 kernel stats of it (averages in us).
#   bash tools/lab_prof.sh TAG "PYTEST -k EXPR or -" CONFIG [bench args...]
set -u
TAG=$1; KEXPR=$2; CFG=$3; shift 3
bash tools/lab_run.sh $TAG "$KEXPR" "$CFG" "$@" || exit 1
OUT=gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --config $CFG --no-cpu --steps 30 --warmup 5 "$@" > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
python -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')):
    if 'anonymous' in r['Name'] and 'k_copy' not in r['Name']:
        print('%-40s %5s avg %9.2f us  min %9.2f' % (r['Name'].split('(')[1].split('::')[-1][:40] if r['Name'].startswith('void') else r['Name'].split('::')[1].split('(')[0], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))
"
