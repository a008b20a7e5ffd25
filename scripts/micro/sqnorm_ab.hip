// Gradient square-norm sweep over the step's flat fp16 gradient (150.45 M values, 301 MB > the
// 256 MB Infinity Cache): the library's mms2ut_grad_sqnorm (C-ABI) against the round-4 kernel kept
// here for the A/B (one 16-B load per thread per iteration).  Checks the 1024 per-block partials
// agree bit for bit, then times 40 launches of each under HIP events.
// Build: hipcc -O3 -w --offload-arch=gfx950 scripts/micro/sqnorm_ab.hip -Lmultimodal-s2ut_amd/lib -lmms2ut_hip
//        -Wl,-rpath,'$ORIGIN/../../multimodal-s2ut_amd/lib' -o scripts/micro/sqnorm_ab
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/mms2ut.h"
#include "../../multimodal-s2ut_amd/csrc/common.h"

__global__ void fill(h16* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
    p[i] = (h16)(((float)(h & 0xffff) / 32768.f - 1.f) * 0.01f);
  }
}

__global__ void sqnorm_old(const h16* __restrict__ g, long n, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const long n8 = n / 8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    h16x8 v = *reinterpret_cast<const h16x8*>(g + i * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float x = (float)v[e]; s += x * x; }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

int main() {
  const long n = 150450000;   // multiple of 8
  const int np = 1024, R = 40;
  h16* g;
  float *pa, *pb;
  hipMalloc(&g, n * 2); hipMalloc(&pa, np * 4); hipMalloc(&pb, np * 4);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, g, n, 3u);
  hipLaunchKernelGGL(sqnorm_old, dim3(np), dim3(256), 0, 0, g, n, pa);
  if (mms2ut_grad_sqnorm(g, n, pb, np, 0)) { printf("launch failed\n"); return 1; }
  hipDeviceSynchronize();
  float ha[1024], hb[1024];
  hipMemcpy(ha, pa, sizeof ha, hipMemcpyDeviceToHost);
  hipMemcpy(hb, pb, sizeof hb, hipMemcpyDeviceToHost);
  // (same wave / block reduction as the library's: the partials must agree bit for bit)
  double md = 0.0;
  int same = 0;
  for (int i = 0; i < np; ++i) {
    same += memcmp(&ha[i], &hb[i], 4) == 0;
    const double d = fabs((double)ha[i] - hb[i]) / fabs((double)ha[i]);
    if (d > md) md = d;
  }
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  float t_old = 0.f, t_new = 0.f;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(a, 0);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(sqnorm_old, dim3(np), dim3(256), 0, 0, g, n, pa);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(&t_old, a, b);
    hipEventRecord(a, 0);
    for (int r = 0; r < R; ++r) mms2ut_grad_sqnorm(g, n, pb, np, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(&t_new, a, b);
    printf("rep %d: old %.2f us (%.3f TB/s), library %.2f us (%.3f TB/s)\n", rep, t_old * 1e3 / R,
           2.0 * n / (t_old * 1e3 / R) / 1e6, t_new * 1e3 / R, 2.0 * n / (t_new * 1e3 / R) / 1e6);
  }
  printf("partials bit-identical %d / %d, max rel diff %.3g\n", same, np, md);
  return 0;
}
