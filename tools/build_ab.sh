#!/bin/bash
# Build an A/B copy of librazor_fec_v1200.so from the product sources with extra
# hipcc defines for one HIP source (container side):
#   [SRC=rfec_kernels] [VS=1000] [SRCFILE=path] bash tools/build_ab.sh <name> -DMACRO=...
#   (SRCFILE: another version of that source, e.g. `git show HEAD~1:razor_amd/csrc/rfec_kernels.hip`)
#   -> tools/bin/ab/librazor_fec[_v1200]_<name>.so (travels to the GPU box, not to git)
set -eu
name=$1; shift
SRC=${SRC:-rfec_wire}
VS=${VS:-1200}   # SIM_VIDEO_SIZE of the host objects: 1200 (wire bench) or 1000 (bench.py)
LIB=librazor_fec_v1200; [ $VS = 1000 ] && LIB=librazor_fec
O=razor_amd/lib/obj; D=tools/bin/ab; mkdir -p $D
SRCFILE=${SRCFILE:-razor_amd/csrc/$SRC.hip}
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Iinclude -Irazor_amd/csrc "$@" -c -x hip "$SRCFILE" -o $D/${SRC}_$name.o
objs=""
for s in rfec_kernels rfec_probe rfec_wire rfec_fill rfec_service rfec_hostio; do
  if [ $s = $SRC ]; then objs="$objs $D/${SRC}_$name.o"; else objs="$objs $O/$s.o"; fi
done
hipcc -shared -fPIC $objs $O/rfec_net.o $O/*_v$VS.o -o $D/${LIB}_$name.so -Wl,-soname,$LIB.so -lpthread -lm
echo built $D/${LIB}_$name.so
