#!/bin/bash
# Build kbench binaries with compile-time variants of library sources (tools/var/kbench_<name>) for
# A/B runs of one kernel family:  tools/kvariants.sh "k_dw_fwd k_dw_strip" name1 "-DFOO=1" name2 "-DFOO=2" ...
# (the named sources are rebuilt with the flags; every other object is the library's own build)
set -e
cd "$(dirname "$0")"
CSRC=../deepfake-video-detection_amd/csrc
SRCS=$1; shift
mkdir -p var
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  objs=$(ls $CSRC/build/*.o)
  for src in $SRCS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -munsafe-fp-atomics $flags \
      -c $CSRC/$src.hip -o var/${src}_$name.o
    objs=$(echo "$objs" | grep -v "/$src.o$")
    objs="$objs var/${src}_$name.o"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -o var/kbench_$name kbench.o $objs -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
done
