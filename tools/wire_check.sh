# wire-codec GPU tests, then the wire bench (+ rocprofv3 stats of it)
set -o pipefail
export TMPDIR=/tmp
T=${1:-wc}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_sender.py tests/test_receiver.py tests/test_udp.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$T/pytest.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/$T/wire.json > gpurun_out/$T/wire.log 2>&1; echo "wire rc=$?"
grep -E "median_us|frac|verified" gpurun_out/$T/wire.json
