#!/bin/bash
# (container) copy a tools/measure.sh pass from gpurun_out/<tag> into profiles/<dir>
#   bash tools/collect_pass.sh r4m4 profiles/r04/m4
set -eu
S=gpurun_out/$1; D=$2; mkdir -p $D
for f in bench bench_c3full bench_c5; do grep '^{' $S/$f.log | tail -1 > $D/$f.json; done
cp $S/group_bench.log $S/smoke.log $S/steps.log $S/traffic_c3.json $S/traffic_c3full.json $S/traffic_c5.json $S/wire.json $D/
[ -f $S/traffic_c5p.json ] && cp $S/traffic_c5p.json $D/
tail -3 $S/pytest_gpu.log > $D/pytest_gpu_tail.txt
grep '^{' $S/mix.log > $D/mix.json
grep '^{' $S/e2e.log > $D/e2e_step.json
cp $S/prof/run_kernel_stats.csv $D/rocprof_kernel_stats_default.csv
cp $S/prof_c3full/run_kernel_stats.csv $D/rocprof_kernel_stats_c3full.csv
cp $S/prof_c5/run_kernel_stats.csv $D/rocprof_kernel_stats_c5.csv
cp $S/prof_wire/run_kernel_stats.csv $D/rocprof_kernel_stats_wire.csv
python3 tools/phase_stats.py $S/prof/run_kernel_trace.csv > $D/kernel_stats_by_phase_default.json
