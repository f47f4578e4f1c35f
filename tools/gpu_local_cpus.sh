#!/bin/bash
# (GPU box) the CPUs of the visible GPU's NUMA node (empty when unknown)
bdf=$(rocm-smi --showbus 2>/dev/null | sed -n 's/.*PCI Bus: *\([0-9A-Fa-f:.]*\).*/\1/p' | head -1 | tr 'A-F' 'a-f')
node=$(cat /sys/bus/pci/devices/$bdf/numa_node 2>/dev/null)
[ -n "$node" ] && [ "$node" -ge 0 ] 2>/dev/null && cat /sys/devices/system/node/node$node/cpulist 2>/dev/null
