# receiver path after a host change: tests, rx_bench, udp_bench (streaming sessions)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rxc
timeout -k 10 600 python -u -m pytest tests/test_receiver.py tests/test_udp.py tests/test_sender.py -q --timeout 120 --timeout-method thread > gpurun_out/rxc/pytest.log 2>&1 || { tail -30 gpurun_out/rxc/pytest.log; exit 1; }
tail -1 gpurun_out/rxc/pytest.log
timeout -k 10 300 python tools/rx_bench.py --out gpurun_out/rxc/rx.json > gpurun_out/rxc/rx.log 2>&1 || exit $?
timeout -k 10 300 python tools/udp_bench.py --out gpurun_out/rxc/udp.json > gpurun_out/rxc/udp.log 2>&1 || exit $?
python - <<'PY'
import json
r=json.load(open('gpurun_out/rxc/rx.json')); u=json.load(open('gpurun_out/rxc/udp.json'))
print('rx', {k: r[k] for k in r if 'per_s' in k or k in ('verified',)})
print('udp', u['recv_datagrams_per_s'], u['streaming']['push_datagrams_per_s'], u['streaming']['batches'], u['ingest_datagrams_per_s'], u.get('verified'))
PY
