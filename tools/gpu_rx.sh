#!/bin/bash
# receiver tests + session push A/B (synchronous vs pipelined, previous build)
set -o pipefail
mkdir -p gpurun_out/rx
timeout -k 10 400 python -u -m pytest tests/test_receiver.py tests/test_udp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rx/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/rx/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
timeout -k 10 200 python tools/session_bench.py --batches 256,1024,4096 --out gpurun_out/rx/sync_$r.json | tail -3 || exit 1
timeout -k 10 200 python tools/session_bench.py --batches 256,1024,4096 --pipelined --out gpurun_out/rx/pipe_$r.json | tail -3 || exit 1
done
