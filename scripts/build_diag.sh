#!/bin/bash
# Diagnostic library (lib/libmms2ut_hip_diag.so): the normal objects, with attention.hip rebuilt
# with -DMMS_ATTN_PHASES (phase stamps of the fused attention backward).  Load it with
# MMS2UT_LIB=multimodal-s2ut_amd/lib/libmms2ut_hip_diag.so (scripts/attn_phases.py).  Run after build.py.
set -e
cd "$(dirname "$0")/../multimodal-s2ut_amd"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -I../include"
$H $F -DMMS_ATTN_PHASES -c csrc/attention.hip -o lib/obj/attention_diag.o
objs=$(ls lib/obj/*.o | grep -v attention)
$H --offload-arch=gfx950 -shared -fPIC $objs lib/obj/attention_diag.o -o lib/libmms2ut_hip_diag.so
echo built lib/libmms2ut_hip_diag.so
