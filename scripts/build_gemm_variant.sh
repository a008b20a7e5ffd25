#!/bin/bash
# A/B build of one csrc file (SRC, default gemm) only, linked with the default build's other objects (lib/obj):
#   [SRC=ops] scripts/build_gemm_variant.sh NAME [-DFOO=1 ...]   -> multimodal-s2ut_amd/lib/libmms2ut_hip_NAME.so
set -e
name=$1; shift
cd "$(dirname "$0")/../multimodal-s2ut_amd"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -I../include"
mkdir -p lib/ab/$name
/opt/rocm/bin/hipcc $F "$@" -c csrc/${SRC:-gemm}.hip -o lib/ab/$name/${SRC:-gemm}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls lib/obj/*.o | grep -v "/${SRC:-gemm}.o$") lib/ab/$name/${SRC:-gemm}.o -o lib/libmms2ut_hip_$name.so
echo built lib/libmms2ut_hip_$name.so
