# one-launch cascade decode (default for plans with columns) vs peel + replay (4096)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_receiver.py tests/test_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cab/pytest.log 2>&1 || { tail -30 gpurun_out/cab/pytest.log; exit 1; }
tail -1 gpurun_out/cab/pytest.log
for rep in 1 2; do
for t in 0 4096; do
  timeout -k 10 300 python bench.py --no-cpu --full-plan --tuning $t --steps 60 > gpurun_out/cab/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/cab/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['decode_roofline']['frac'], d['verified'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cab/prof -o run -- python bench.py --no-cpu --full-plan --steps 20 > gpurun_out/cab/prof.log 2>&1; echo prof rc=$?
