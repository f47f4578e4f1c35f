# matrix-plan encode: parity tests touching full plans, then the full-plan bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mx
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "sender or full_size or erasure_fixture_gpu" > gpurun_out/mx/pytest.log 2>&1 || { tail -30 gpurun_out/mx/pytest.log; exit 1; }
tail -3 gpurun_out/mx/pytest.log
for t in 0 64 4; do
  timeout -k 10 300 python bench.py --no-cpu --full-plan --tuning $t --steps 50 > gpurun_out/mx/t$t.log 2>&1 || exit $?
  grep '^{' gpurun_out/mx/t$t.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us'], d['roofline']['frac'], d['decode_roofline']['launch_us'], d['verified'])"
done
timeout -k 10 300 python bench.py --no-cpu --steps 50 > gpurun_out/mx/c2.log 2>&1 && grep '^{' gpurun_out/mx/c2.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mx/prof -o run -- python bench.py --no-cpu --full-plan --steps 20 > gpurun_out/mx/prof.log 2>&1; echo prof rc=$?
