#!/bin/bash
# A/B build of gemm.hip only, linked with the default build's other objects (lib/obj):
#   scripts/build_gemm_variant.sh NAME [-DFOO=1 ...]   -> multimodal-s2ut_amd/lib/libmms2ut_hip_NAME.so
set -e
name=$1; shift
cd "$(dirname "$0")/../multimodal-s2ut_amd"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -I../include"
mkdir -p lib/ab/$name
/opt/rocm/bin/hipcc $F "$@" -c csrc/gemm.hip -o lib/ab/$name/gemm.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls lib/obj/*.o | grep -v '/gemm.o$') lib/ab/$name/gemm.o -o lib/libmms2ut_hip_$name.so
echo built lib/libmms2ut_hip_$name.so
