# GPU box: the receiver tests, then tools/gcmd_rx.sh.  bash tools/g_rx_check.sh <tag>
set -o pipefail
TAG=${1:-rx}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_receiver.py tests/test_udp.py tests/test_rx_shards.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_rx.log 2>&1 && RFEC_RX_TRACE=1 bash tools/gcmd_rx.sh $TAG
