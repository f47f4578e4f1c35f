set -o pipefail
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_receiver.py tests/test_udp.py > gpurun_out/t_rx.log 2>&1 && \
timeout -k 10 400 python -u tools/rx_session_bench.py --frames 32768 --threads 1,4,8,16 --out gpurun_out/rxs2.json > gpurun_out/rxs2.log 2>&1 && \
for t in 1 2 4 8 16; do timeout -k 10 120 python -u tools/rx_host_bench.py --groups 65536 --no-verify --lib tools/bin/librazor_fec_rxhost.so --threads $t >> gpurun_out/rxh.log 2>&1 || exit 1; done
