#!/bin/bash
# service A/B call (GPU box): service / drop-in GPU tests, then tools/svc_ab.sh over the product,
# the previous build (tools/bin/ab/prev) and the product with the request side in host memory
set -u
mkdir -p gpurun_out/svc
timeout -k 10 300 python -u -m pytest tests/test_service.py tests/test_flex_dropin.py tests/test_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/svc/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/svc/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/svc_ab.sh "${SVC_VARIANTS:-prev env:RFEC_SERVICE_STAGE=host}" ${SVC_ROUNDS:-3} 2>&1 | tee gpurun_out/svc/ab.txt
[ -x tools/bin/sclk_probe ] && timeout -k 10 60 ./tools/bin/sclk_probe | tee gpurun_out/svc/sclk.json
