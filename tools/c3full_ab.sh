# full-plan (config 3 variant) store policies: default / NT (512) / plain (4) / WT+NT (192), then rocprofv3 stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c3ab
for t in 0 512 4 192; do
  timeout -k 10 300 python bench.py --no-cpu --full-plan --tuning $t --steps 50 > gpurun_out/c3ab/t$t.log 2>&1 || exit $?
  grep '^{' gpurun_out/c3ab/t$t.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us'], d['decode_roofline']['launch_us'], d['verified'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3ab/prof -o run -- python bench.py --no-cpu --full-plan --steps 20 > gpurun_out/c3ab/prof.log 2>&1; echo prof rc=$?
