#!/bin/bash
# Wire-kernel cost breakdown: build (container) or run (GPU box) the lab variants.
#   bash tools/wire_lab.sh build      # here: hipcc, tools/bin/wire_lab_*
#   bash tools/wire_lab.sh run        # GPU box
set -u
V="base: nocrc:-DRFEC_WIRE_DIAG_NO_CRC nocrc_nostore:-DRFEC_WIRE_DIAG_NO_CRC_-DRFEC_WIRE_DIAG_NO_STORE loadonly:-DRFEC_WIRE_DIAG_LOAD_ONLY nopass1:-DRFEC_WIRE_DIAG_NO_PASS1 pass1_noload:-DRFEC_WIRE_DIAG_PASS1_NOLOAD"
if [ "${1:-run}" = build ]; then
  # the product source with the measurement-only RFEC_WIRE_DIAG_* switches patched in (tools/wire_lab.patch)
  mkdir -p tools/bin/wire_lab_src
  cp razor_amd/csrc/rfec_wire.hip tools/bin/wire_lab_src/rfec_wire.hip
  patch -s tools/bin/wire_lab_src/rfec_wire.hip tools/wire_lab.patch || exit 1
  for v in $V; do
    name=${v%%:*}; flags=${v#*:}; flags=${flags//_-D/ -D}
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Irazor_amd/csrc $flags tools/wire_lab.hip -o tools/bin/wire_lab_$name &
  done
  wait
  ls -la tools/bin/wire_lab_*
else
  mkdir -p gpurun_out/wire_lab
  for round in 1 2; do
    for v in $V; do
      name=${v%%:*}
      echo -n "$name: "; timeout -k 10 120 tools/bin/wire_lab_$name 20 || exit 1
    done
  done | tee gpurun_out/wire_lab/out.txt
fi
