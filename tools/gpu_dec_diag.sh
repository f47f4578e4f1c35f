set -o pipefail
mkdir -p gpurun_out/dec
for r in 1 2; do
for t in 0 1048576 256; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-verify --tuning $t > gpurun_out/dec/t${t}_$r.log 2>&1 || exit 1
python -c "
import json,sys
d=json.loads(open('gpurun_out/dec/t${t}_$r.log').read().strip().splitlines()[-1])
print('tuning', $t, 'value', d['value'], 'enc', d['roofline']['launch_us'], 'dec', d['decode_roofline']['launch_us'])
"
done; done
