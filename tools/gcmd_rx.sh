# GPU box: host-plane sweep (stub lib, the box's CPUs), session bench sweep
set -o pipefail
for t in 1 4 8 16; do timeout -k 10 120 python -u tools/rx_host_bench.py --groups 65536 --no-verify --lib tools/bin/librazor_fec_rxhost.so --threads $t >> gpurun_out/rxh.log 2>&1 || exit 1; done && \
RFEC_RX_ARENA_ROWS=1048576 timeout -k 10 400 python -u tools/rx_session_bench.py --frames 32768 --threads 1,8,16 --modes async,sync --out gpurun_out/rxs4.json > gpurun_out/rxs4.log 2>&1
