# secondary configurations with rotated buffer sets
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cfgrot
timeout -k 10 300 python bench.py --no-cpu --full-plan --steps 60 > gpurun_out/cfgrot/c3full.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --k 32 --payload 256 --col 4 --steps 60 > gpurun_out/cfgrot/c5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 60 > gpurun_out/cfgrot/c2.log 2>&1 || exit $?
for c in c3full c5 c2; do grep '^{' gpurun_out/cfgrot/$c.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['roofline']['launch_us_median'], d['roofline']['frac'], d['decode_roofline']['launch_us_median'], d['decode_roofline']['frac'], d['verified'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfgrot/prof -o run -- python bench.py --no-cpu --full-plan --steps 20 > gpurun_out/cfgrot/prof.log 2>&1; echo prof rc=$?
