#!/bin/bash
# GPU box: the receive path after a wire-kernel change: the session bench at 4,096 / 16,384-datagram batches
# and the session soak against the oracle.  bash tools/g_rx_soak.sh <tag>
set -u
TAG=${1:-rxs}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
LOCAL=$(bash tools/gpu_local_cpus.sh); PIN=(); [ -n "$LOCAL" ] && PIN=(taskset -c "$LOCAL")
timeout -k 10 300 "${PIN[@]}" python -u tools/rx_session_bench.py --frames 32768 --threads 8 --batch 4096 --modes async --reps 3 --out "$OUT/rx_b4096.json" > "$OUT/rx_b4096.log" 2>&1 || { tail -20 "$OUT/rx_b4096.log"; exit 1; }
tail -3 "$OUT/rx_b4096.log"
timeout -k 10 300 "${PIN[@]}" python -u tools/rx_session_bench.py --frames 32768 --threads 8 --batch 16384 --modes async --reps 3 --out "$OUT/rx_b16384.json" > "$OUT/rx_b16384.log" 2>&1 || { tail -20 "$OUT/rx_b16384.log"; exit 1; }
tail -3 "$OUT/rx_b16384.log"
timeout -k 10 300 "${PIN[@]}" python -u tools/soak_rx.py --seconds ${SOAK_S:-150} --out "$OUT/soak_rx.json" > "$OUT/soak_rx.log" 2>&1 || { tail -20 "$OUT/soak_rx.log"; exit 1; }
tail -3 "$OUT/soak_rx.log"
