#!/bin/bash
# Whole-library A/B build: every csrc/*.hip recompiled under extra -D flags (for switches in shared
# headers, e.g. the dropout mixer in common.h).
#   scripts/build_variant.sh NAME [-DFOO=1 ...]   -> multimodal-s2ut_amd/lib/libmms2ut_hip_NAME.so
# Load it with MMS2UT_LIB=multimodal-s2ut_amd/lib/libmms2ut_hip_NAME.so.
set -e
name=$1; shift
cd "$(dirname "$0")/../multimodal-s2ut_amd"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -I../include"
mkdir -p lib/ab/$name
ls csrc/*.hip | xargs -P 8 -I{} sh -c "/opt/rocm/bin/hipcc $F $* -c {} -o lib/ab/$name/\$(basename {} .hip).o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC lib/ab/$name/*.o -o lib/libmms2ut_hip_$name.so
echo built lib/libmms2ut_hip_$name.so
