#!/bin/bash
# A/B library builds: libdfd_hip_<tag>.so = the in-tree objects with one source (default k_vgemm)
# recompiled under extra defines (tools/ab_lib.sh xp1 -DDFD_VG_XP_DEFAULT=1, or
# SRC=k_resnet tools/ab_lib.sh pf0 -DDFD_RSTEM_PF=0); load it with DFD_HIP_LIB=<path>.
set -e
TAG=$1; shift
SRC=${SRC:-k_vgemm}
C=$(cd "$(dirname "$0")/../deepfake-video-detection_amd/csrc" && pwd)
mkdir -p $C/build_ab
SF=$C/$SRC.hip; XL=""
[ -f $SF ] || { SF=$C/$SRC.cpp; XL="-x hip"; }  # host sources (plan.cpp, vit.cpp) build as HIP too
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 \
  -fvisibility=hidden -munsafe-fp-atomics "$@" $XL -c $SF -o $C/build_ab/${SRC}_$TAG.o
OBJS=$(ls $C/build/*.o | grep -v "/$SRC.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $C/../libdfd_hip_$TAG.so.tmp $OBJS $C/build_ab/${SRC}_$TAG.o \
  -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
mv -f $C/../libdfd_hip_$TAG.so.tmp $C/../libdfd_hip_$TAG.so
echo built $C/../libdfd_hip_$TAG.so
