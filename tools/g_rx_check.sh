set -o pipefail
mkdir -p gpurun_out/rx2
timeout -k 10 600 python -u -m pytest tests/test_receiver.py tests/test_udp.py tests/test_rx_shards.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rx2/pytest_rx.log 2>&1 && RFEC_RX_TRACE=1 bash tools/gcmd_rx.sh rx2
