#!/bin/bash
# The paths around the device path that start / end in host memory: end to end from sim_segment_t arrays,
# sender staging, receiver ingestion, loopback UDP into receiver sessions, pipelined session pushes.
set -u
OUT=gpurun_out/${1:-hp}; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 300 python "$@" --out $OUT/$name.json > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; exit 1; }
  echo "$name ok"; }
run e2e tools/e2e_bench.py
run send tools/send_bench.py
run rx tools/rx_bench.py
run udp tools/udp_bench.py
timeout -k 10 300 python tools/session_bench.py --pipelined --out $OUT/session_pipe.json > $OUT/session_pipe.log 2>&1 || { tail $OUT/session_pipe.log; exit 1; }
echo done
