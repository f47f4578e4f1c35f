# encode header work: LDS-staged meta blocks (default) vs one lane per (group, line) (65536), rotated sets
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sender and meta_lines" > gpurun_out/mab/pytest.log 2>&1 || { tail -30 gpurun_out/mab/pytest.log; exit 1; }
tail -1 gpurun_out/mab/pytest.log
for rep in 1 2 3; do
for t in 0 65536; do
  timeout -k 10 300 python bench.py --no-cpu --tuning $t --steps 60 > gpurun_out/mab/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/mab/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
for t in 0 65536; do
  timeout -k 10 300 python bench.py --no-cpu --full-plan --tuning $t --steps 60 > gpurun_out/mab/f$t.log 2>&1 || exit $?
  grep '^{' gpurun_out/mab/f$t.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('full tuning $t', d['value'], d['roofline']['launch_us_median'], d['verified'])"
done
