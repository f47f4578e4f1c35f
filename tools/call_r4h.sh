#!/bin/bash
# (GPU box) host-recover packing check + e2e step, then the service A/B
set -u
mkdir -p gpurun_out/r4h
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "host_recover" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4h/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4h/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/e2e_step.py > gpurun_out/r4h/e2e.json 2> gpurun_out/r4h/e2e.err
rc=$?; tail -c 1500 gpurun_out/r4h/e2e.json; [ $rc -ne 0 ] && exit $rc
SVC_VARIANTS="${SVC_VARIANTS:-pin:local svc_b4+pin:local svc_b8+pin:local}" SVC_ROUNDS=3 bash tools/call_svc.sh
