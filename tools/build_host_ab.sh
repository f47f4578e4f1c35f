#!/bin/bash
# (container) An A/B copy of librazor_fec_v1200.so whose host layer comes from another rfec_host.c
# (e.g. a patched copy), into tools/bin/ab/<name>/ for tools/svc_ab.sh:
#   bash tools/build_host_ab.sh <name> <rfec_host.c>
set -eu
name=$1; src=$2
O=razor_amd/lib/obj; D=tools/bin/ab/$name; mkdir -p $D
gcc -std=c99 -O2 -fPIC -Wall -Wextra -Wno-unused-parameter -DSIM_VIDEO_SIZE=1200 -D__HIP_PLATFORM_AMD__ \
    -I/opt/rocm/include -Iinclude -Irazor_amd/csrc -c "$src" -o $D/rfec_host_v1200.o
hipcc -shared -fPIC $O/rfec_kernels.o $O/rfec_probe.o $O/rfec_wire.o $O/rfec_fill.o $O/rfec_service.o $O/rfec_net.o \
    $D/rfec_host_v1200.o $O/rfec_flex_v1200.o -o $D/librazor_fec_v1200.so -Wl,-soname,librazor_fec_v1200.so -lpthread -lm
echo built $D/librazor_fec_v1200.so
