#!/bin/bash
# Build an A/B copy of librazor_fec_v1200.so from the product sources with extra
# hipcc defines for rfec_wire.hip (container side):
#   bash tools/build_ab.sh <name> -DMACRO=...   -> tools/bin/ab/librazor_fec_v1200_<name>.so (travels to the GPU box, not to git)
set -eu
name=$1; shift
O=razor_amd/lib/obj; D=tools/bin/ab; mkdir -p $D
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Iinclude -Irazor_amd/csrc "$@" -c razor_amd/csrc/rfec_wire.hip -o $D/rfec_wire_$name.o
hipcc -shared -fPIC $O/rfec_kernels.o $O/rfec_probe.o $D/rfec_wire_$name.o $O/rfec_fill.o $O/rfec_net.o $O/*_v1200.o \
  -o $D/librazor_fec_v1200_$name.so -Wl,-soname,librazor_fec_v1200.so -lpthread -lm
echo built $D/librazor_fec_v1200_$name.so
