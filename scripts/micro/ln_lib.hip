// LayerNorm kernels of the library (C-ABI, no Python in the loop) on the encoder shape, 10000 x 768:
// back-to-back launches over NSET rotating buffer sets (NSET x 77 MB > the 256 MB Infinity Cache,
// so every launch streams from HBM), HIP events around 60 launches.  Also the same launches on ONE
// buffer set (cache-warm), for comparison with scripts/micro/ln_stream.
// Build: hipcc -O3 -w --offload-arch=gfx950 scripts/micro/ln_lib.hip -Lmultimodal-s2ut_amd/lib -lmms2ut_hip
//        -Wl,-rpath,'$ORIGIN/../../multimodal-s2ut_amd/lib' -o scripts/micro/ln_lib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/mms2ut.h"

typedef _Float16 h16;
constexpr int D = 768, NSET = 6;
constexpr long ROWS = 10000;

__global__ void fill(h16* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
    p[i] = (h16)(((float)(h & 0xffff) / 32768.f - 1.f));
  }
}

struct Set {
  h16 *x, *dy, *dres, *dx, *dxd, *y;
  float *mean, *rstd, *part;
};

int main() {
  const long n = ROWS * D;
  h16 *g, *b;
  hipMalloc(&g, D * 2); hipMalloc(&b, D * 2);
  hipLaunchKernelGGL(fill, dim3(4), dim3(256), 0, 0, g, (long)D, 7u);
  hipLaunchKernelGGL(fill, dim3(4), dim3(256), 0, 0, b, (long)D, 9u);
  Set s[NSET];
  const int np = mms2ut_layernorm_bwd_nparts(ROWS, D);
  for (int i = 0; i < NSET; ++i) {
    hipMalloc(&s[i].x, n * 2); hipMalloc(&s[i].dy, n * 2); hipMalloc(&s[i].dres, n * 2);
    hipMalloc(&s[i].dx, n * 2); hipMalloc(&s[i].dxd, n * 2); hipMalloc(&s[i].y, n * 2);
    hipMalloc(&s[i].mean, ROWS * 4); hipMalloc(&s[i].rstd, ROWS * 4); hipMalloc(&s[i].part, (size_t)np * 2 * D * 4);
    hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, s[i].x, n, 11u + i);
    hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, s[i].dy, n, 23u + i);
    hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, s[i].dres, n, 37u + i);
    mms2ut_layernorm_fwd(s[i].x, g, b, s[i].y, s[i].mean, s[i].rstd, ROWS, D, 1e-5f, 0);
  }
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, double mb, int nset, auto launch) {
    for (int i = 0; i < 6; ++i) launch(s[i % nset]);
    hipEventRecord(e0);
    constexpr int R = 60;
    for (int i = 0; i < R; ++i) launch(s[i % nset]);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / R;
    printf("%-40s %s %7.1f us  %6.0f GB/s (%.1f MB)\n", name, nset > 1 ? "cold" : "warm", us, mb * 1e3 / us, mb);
  };
  const double mb = n * 2 / 1e6;
  for (int nset : {NSET, 1}) {
    run("layernorm_fwd", 2 * mb, nset, [&](Set& t) {
      mms2ut_layernorm_fwd(t.x, g, b, t.y, t.mean, t.rstd, ROWS, D, 1e-5f, 0);
    });
    run("layernorm_bwd (+dres)", 4 * mb, nset, [&](Set& t) {
      mms2ut_layernorm_bwd(t.dy, t.x, g, t.mean, t.rstd, t.dres, t.dx, t.part, ROWS, D, nullptr, 0.f, 0, 0, 0);
    });
    run("layernorm_bwd (+dres, emit drop)", 5 * mb, nset, [&](Set& t) {
      mms2ut_layernorm_bwd(t.dy, t.x, g, t.mean, t.rstd, t.dres, t.dx, t.part, ROWS, D, t.dxd, 0.1f, 1, 0, 0);
    });
    run("copy x -> dx (hipMemcpyAsync)", 2 * mb, nset, [&](Set& t) {
      hipMemcpyAsync(t.dx, t.x, n * 2, hipMemcpyDeviceToDevice, 0);
    });
  }
  printf("rc %s\n", mms2ut_last_error());
  return 0;
}
