#!/bin/bash
# The drop-in's resident service on the GPU box: the drop-in GPU tests (service, relaunch and
# per-call-launch modes), then the per-group drop-in cost with the service and without it.
#   bash tools/svc_check.sh TAG
set -u
TAG=${1:-svc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_flex_dropin.py tests/test_dropin.py -x -v -m gpu \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 120 ./razor_amd/lib/fec_dropin_group_bench 2000 > "$OUT/group_service.json" || exit 1
RFEC_SERVICE=0 timeout -k 10 120 ./razor_amd/lib/fec_dropin_group_bench 2000 > "$OUT/group_launch.json" || exit 1
RFEC_SERVICE_IDLE_US=1 timeout -k 10 120 ./razor_amd/lib/fec_dropin_group_bench 500 > "$OUT/group_relaunch.json" || exit 1
cat "$OUT"/group_*.json
