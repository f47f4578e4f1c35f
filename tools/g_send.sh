# GPU box: sender tests + send_bench variants.  bash tools/g_send.sh <tag>
set -o pipefail
TAG=${1:-send}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
LOCAL=$(bash tools/gpu_local_cpus.sh)
PIN=(); [ -n "$LOCAL" ] && PIN=(taskset -c "$LOCAL")
timeout -k 10 300 python -u -m pytest tests/test_sender.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_send.log 2>&1 &&
timeout -k 10 200 "${PIN[@]}" python tools/send_bench.py --out $OUT/send_zc.json > $OUT/send_zc.log 2>&1 &&
timeout -k 10 200 "${PIN[@]}" python tools/send_bench.py --frames-mem pageable --out $OUT/send_outzc.json > $OUT/send_outzc.log 2>&1 &&
RFEC_HOST_ZEROCOPY=0 timeout -k 10 200 "${PIN[@]}" python tools/send_bench.py --out $OUT/send_staged.json > $OUT/send_staged.log 2>&1 &&
timeout -k 10 200 "${PIN[@]}" python tools/send_bench.py --chunk 65536 --out $OUT/send_zc_big.json > $OUT/send_zc_big.log 2>&1
