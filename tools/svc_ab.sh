#!/bin/bash
# A/B of drop-in service builds (GPU box): tools/dropin_group_bench.c against the product library and
# against variants.  A variant is a '+'-joined list of:
#   <dir>        tools/bin/ab/<dir>/librazor_fec_v1200.so (LD_LIBRARY_PATH overrides the bench's RUNPATH)
#   env:VAR=val  an environment setting
#   pin:local    the bench pinned to the CPUs of the visible GPU's NUMA node; pin:remote the other node's
#   cur          the product library, unpinned
# Prints: variant round outputs_equal, mean / median sender and on_segment us, sender p10, service phases.
#   bash tools/svc_ab.sh "name1 pin:local cur+pin:remote ..." [rounds]
set -u
VARIANTS=${1:-}; R=${2:-2}
mkdir -p gpurun_out/svcab
bdf=$(rocm-smi --showbus 2>/dev/null | sed -n 's/.*PCI Bus: *\([0-9A-Fa-f:.]*\).*/\1/p' | head -1 | tr 'A-F' 'a-f')
node=$(cat /sys/bus/pci/devices/$bdf/numa_node 2>/dev/null || echo -1)
cpus_of() { cat /sys/devices/system/node/node$1/cpulist 2>/dev/null; }
other=$(( node == 0 ? 1 : 0 ))
echo "gpu $bdf numa node $node; local cpus $(cpus_of $node); remote cpus $(cpus_of $other)"
for r in $(seq 1 "$R"); do
  for v in cur $VARIANTS; do
    LP=""; EV=""; PIN=""
    for t in ${v//+/ }; do
      case "$t" in
        cur) ;;
        env:*) EV="$EV ${t#env:}" ;;
        pin:local) PIN="taskset -c $(cpus_of $node)" ;;
        pin:remote) PIN="taskset -c $(cpus_of $other)" ;;
        *) LP="tools/bin/ab/$t" ;;
      esac
    done
    f="gpurun_out/svcab/${v//[:=+]/_}.$r.json"
    env $EV LD_LIBRARY_PATH=$LP timeout -k 10 60 $PIN ./razor_amd/lib/fec_dropin_group_bench 2000 > "$f"
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$v: rc=$rc"; exit $rc; fi  # 1: outputs differ (reported)
    python3 - "$v" "$r" "$f" <<'PY'
import json, sys
v, r, f = sys.argv[1:4]
d = json.load(open(f))
s = d["service_sender"]
print(v, r, d["outputs_equal"], "mean", d["sender_group_level_us_per_group"], d["receiver_on_segment_row_and_col_us"],
      "median", d.get("sender_group_level_us_median"), d.get("receiver_on_segment_us_median"),
      "p10", d.get("sender_group_level_us_p10"),
      "| wait", s["wait_us"], s["dev_stage_us"], s["dev_work_us"], s["dev_release_us"], s.get("request_in_device"))
PY
  done
done
