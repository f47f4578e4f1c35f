# secondary bench configurations (BASELINE configs 3b and 5) + the headline for reference, same box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/cfg/c3.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --full-plan > gpurun_out/cfg/c3full.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --k 32 --payload 256 --col 4 > gpurun_out/cfg/c5.log 2>&1
echo rc=$?
for f in c3 c3full c5; do grep '^{' gpurun_out/cfg/$f.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['config']['plan'], d['roofline']['kernel'], d['roofline']['launch_us'], d['roofline']['frac'], d['decode_roofline']['launch_us'], d['decode_roofline']['frac'], d['verified'])"; done
