#!/bin/bash
# The drop-in service's per-group cost by workgroup count (GPU box):
#   bash tools/svc_groups.sh TAG [rounds]
set -u
TAG=${1:-svcg}; R=${2:-2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for g in 1 2 4 8; do
    RFEC_SERVICE_GROUPS=$g timeout -k 10 60 ./razor_amd/lib/fec_dropin_group_bench 2000 > "$OUT/g$g.$r.json" || exit 1
    python3 - "$OUT/g$g.$r.json" "$g" "$r" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); s = d["service_sender"]
print("groups", sys.argv[2], "round", sys.argv[3], d["outputs_equal"], "sender", d["sender_group_level_us_per_group"],
      "line", d["sender_line_level_us_per_group"], "rx", d["receiver_on_segment_row_and_col_us"],
      "wait", s["wait_us"], "stage", s["dev_stage_us"], "work", s["dev_work_us"], "release", s["dev_release_us"])
PY
  done
done
