#!/bin/bash
# (GPU box) where the visible GPU sits relative to this process's CPUs, and the drop-in group bench pinned
# to CPUs of each NUMA node it may use
set -u
mkdir -p gpurun_out/numa
{
echo "allowed: $(taskset -pc $$ 2>/dev/null)"
echo "nproc: $(nproc)"
rocm-smi --showbus 2>/dev/null | grep -i "bus\|GPU\[" | head -8
for d in /sys/class/drm/card*/device; do
  [ -f $d/vendor ] || continue
  [ "$(cat $d/vendor)" = 0x1002 ] || continue
  echo "$(readlink -f $d | xargs basename) numa=$(cat $d/numa_node 2>/dev/null) cpus=$(cat $d/local_cpulist 2>/dev/null)"
done
for n in /sys/devices/system/node/node*; do echo "$(basename $n) cpus=$(cat $n/cpulist)"; done
} 2>&1 | tee gpurun_out/numa/topo.txt
