#!/bin/bash
# A/B of drop-in service builds (GPU box): tools/dropin_group_bench.c against the product library and
# against each variant directory tools/bin/ab/<name>/librazor_fec_v1200.so (LD_LIBRARY_PATH overrides the
# bench's RUNPATH).  Prints: variant round outputs_equal sender_us on_segment_us wait stage work release.
#   bash tools/svc_ab.sh "name1 name2 ..." [rounds]
set -u
VARIANTS=${1:-}; R=${2:-2}
mkdir -p gpurun_out/svcab
for r in $(seq 1 "$R"); do
  for v in cur $VARIANTS; do
    LP=""; EV=""; case "$v" in cur) ;; env:*) EV=${v#env:} ;; *) LP="tools/bin/ab/$v" ;; esac
    env $EV LD_LIBRARY_PATH=$LP timeout -k 10 60 ./razor_amd/lib/fec_dropin_group_bench 2000 > "gpurun_out/svcab/$v.$r.json"
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$v: rc=$rc"; exit $rc; fi  # 1: outputs differ (reported)
    python3 - "$v" "$r" <<'PY'
import json, sys
v, r = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/svcab/{v}.{r}.json"))
s = d["service_sender"]
print(v, r, d["outputs_equal"], d["sender_group_level_us_per_group"], d["receiver_on_segment_row_and_col_us"],
      s["wait_us"], s["dev_stage_us"], s["dev_work_us"], s["dev_release_us"], s.get("request_in_device"))
PY
  done
done
