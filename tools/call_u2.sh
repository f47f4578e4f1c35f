#!/bin/bash
set -u
mkdir -p gpurun_out/u2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/u2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/u2/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/u2/smoke.log 2>&1 || { tail -5 gpurun_out/u2/smoke.log; exit 1; }
bash tools/abn.sh u2ab 4 - tools/bin/ab/librazor_fec_u1.so -- --config c3full --c4-steps 0
