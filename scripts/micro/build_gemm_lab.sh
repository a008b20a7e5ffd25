#!/bin/bash
# Build the GEMM lab (scripts/micro/gemm_lab.hip) against the in-tree library.
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-function -I../../include "$@" \
  gemm_lab.hip -o gemm_lab -L../../multimodal-s2ut_amd/lib -lmms2ut_hip -Wl,-rpath,'$ORIGIN/../../multimodal-s2ut_amd/lib'
echo built scripts/micro/gemm_lab
