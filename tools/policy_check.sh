# encode store default by slot alignment: c5 (256 B), c2 at 1200 / 1280 B strides, WT (64) vs NT (512)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pol
run() { timeout -k 10 300 python bench.py --no-cpu --steps 60 "$@" > gpurun_out/pol/run.log 2>&1 || exit $?; grep '^{' gpurun_out/pol/run.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"; }
for rep in 1 2; do
run --k 32 --payload 256 --col 4
run --stride 1280 --tuning 0
run --stride 1280 --tuning 64
run --tuning 0
done
