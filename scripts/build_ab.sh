#!/bin/bash
# A/B library: the normal objects with ONE source rebuilt under extra -D flags.
#   scripts/build_ab.sh NAME SOURCE.hip [-DFOO=1 ...]   -> multimodal-s2ut_amd/lib/libmms2ut_hip_NAME.so
# Load it with MMS2UT_LIB=multimodal-s2ut_amd/lib/libmms2ut_hip_NAME.so.  Run after build.py.
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../multimodal-s2ut_amd"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -I../include"
base=${src%.hip}
mkdir -p lib/ab
$H $F "$@" -c csrc/$src -o lib/ab/${base}_$name.o
objs=$(ls lib/obj/*.o | grep -v "/$base.o")
$H --offload-arch=gfx950 -shared -fPIC $objs lib/ab/${base}_$name.o -o lib/libmms2ut_hip_$name.so
echo built lib/libmms2ut_hip_$name.so
