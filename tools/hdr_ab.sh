# fused decode header work: line lanes (default) vs LDS peel blocks (32768), c2 and c5
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hdr
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_receiver.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/hdr/pytest.log 2>&1 || { tail -30 gpurun_out/hdr/pytest.log; exit 1; }
tail -2 gpurun_out/hdr/pytest.log
for rep in 1 2; do
for cfg in c2 c5; do
for t in 0 32768; do
  if [ $cfg = c5 ]; then A="--k 32 --payload 256 --col 4"; else A=""; fi
  timeout -k 10 300 python bench.py --no-cpu --tuning $t --steps 50 $A > gpurun_out/hdr/$cfg.t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/hdr/$cfg.t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$cfg tuning $t', d['value'], d['roofline']['launch_us'], d['decode_roofline']['launch_us'], d['decode_roofline']['frac'], d['verified'])"
done; done; done
