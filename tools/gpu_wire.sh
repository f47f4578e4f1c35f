#!/bin/bash
# wire kernels: parity tests, lab breakdown, wire bench
mkdir -p gpurun_out/wire2
timeout -k 10 600 python -u -m pytest tests/test_wire.py tests/test_sender.py tests/test_receiver.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wire2/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/wire2/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 bash tools/wire_lab.sh run; echo lab rc=$?
timeout -k 10 300 python tools/wire_bench.py --out gpurun_out/wire2/wire.json > gpurun_out/wire2/wire.log 2>&1; echo wb rc=$?; tail -30 gpurun_out/wire2/wire.log | grep -E "frac|median|kernels|frame|parse" | head -30
