// Micro-study of the LayerNorm-backward access pattern (rows of D = 768 fp16, 3 row operands read,
// 1-2 written): how fast can a kernel with that shape stream, and what does each piece cost?
//   V0 copy, half-wave per row (the ln_bwd16 mapping), 8 rows per 256-thread block
//   V1 V0 + the two half-wave row reductions (10 shuffles)
//   V2 copy, one wave per row (3 x 8-B per lane), 4 rows per block
//   V3 copy, half-wave per row, 16 rows per block (2 rows per half-wave, all loads issued first)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/ln_stream.hip -o scripts/micro/ln_stream
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 h16;
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
constexpr int D = 768;

template <bool RED>
__global__ void __launch_bounds__(256) v_half(const h16* __restrict__ a, const h16* __restrict__ b,
                                              const h16* __restrict__ c, h16* __restrict__ o, long rows) {
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const long row = (long)blockIdx.x * 8 + (threadIdx.x >> 6) * 2 + (lane >> 5);
  if (row >= rows) return;
  h16x8 x[3], y[3], z[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const long off = row * D + (hl + 32 * k) * 8;
    x[k] = *reinterpret_cast<const h16x8*>(a + off);
    y[k] = *reinterpret_cast<const h16x8*>(b + off);
    z[k] = *reinterpret_cast<const h16x8*>(c + off);
  }
  float s1 = 0.f, s2 = 0.f;
  if (RED) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1 += (float)x[k][e] * (float)y[k][e]; s2 += (float)y[k][e]; }
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) { s1 += __shfl_xor(s1, off, 64); s2 += __shfl_xor(s2, off, 64); }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    h16x8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = (h16)((float)x[k][e] * s1 + (float)y[k][e] - s2 + (float)z[k][e]);
    *reinterpret_cast<h16x8*>(o + row * D + (hl + 32 * k) * 8) = r;
  }
}

__global__ void __launch_bounds__(256) v_wave(const h16* __restrict__ a, const h16* __restrict__ b,
                                              const h16* __restrict__ c, h16* __restrict__ o, long rows) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  h16x4 x[3], y[3], z[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const long off = row * D + (lane + 64 * k) * 4;
    x[k] = *reinterpret_cast<const h16x4*>(a + off);
    y[k] = *reinterpret_cast<const h16x4*>(b + off);
    z[k] = *reinterpret_cast<const h16x4*>(c + off);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    h16x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = (h16)((float)x[k][e] + (float)y[k][e] + (float)z[k][e]);
    *reinterpret_cast<h16x4*>(o + row * D + (lane + 64 * k) * 4) = r;
  }
}

__global__ void __launch_bounds__(256) v_half2(const h16* __restrict__ a, const h16* __restrict__ b,
                                               const h16* __restrict__ c, h16* __restrict__ o, long rows) {
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const long row0 = (long)blockIdx.x * 16 + (threadIdx.x >> 6) * 2 + (lane >> 5);
  h16x8 x[2][3], y[2][3], z[2][3];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const long row = row0 + 8 * q;
      const long off = (row < rows ? row : 0) * D + (hl + 32 * k) * 8;
      x[q][k] = *reinterpret_cast<const h16x8*>(a + off);
      y[q][k] = *reinterpret_cast<const h16x8*>(b + off);
      z[q][k] = *reinterpret_cast<const h16x8*>(c + off);
    }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const long row = row0 + 8 * q;
    if (row >= rows) continue;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      h16x8 r;
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = (h16)((float)x[q][k][e] + (float)y[q][k][e] + (float)z[q][k][e]);
      *reinterpret_cast<h16x8*>(o + row * D + (hl + 32 * k) * 8) = r;
    }
  }
}


// V5: the LayerNorm-backward arithmetic (ln_bwd16_kernel, NP = 1, C8 = 3, no dropout) with switches:
// ACC = dgamma / dbeta accumulation + the block's LDS fold and partial-row store; ITERS row groups
// of 8 per block
template <bool ACC, int ITERS>
__global__ void __launch_bounds__(256) v_ln(const h16* __restrict__ dy, const h16* __restrict__ x,
                                            const h16* __restrict__ dres, const h16* __restrict__ g,
                                            const float* __restrict__ mean, const float* __restrict__ rstd,
                                            h16* __restrict__ dx, float* __restrict__ part, long rows) {
  constexpr int C8 = 3;
  __shared__ __attribute__((aligned(16))) float red[4][2][C8 * 256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5, hl = lane & 31;
  const float invD = 1.f / D;
  float gam[C8][8], dg[C8][8], db[C8][8];
#pragma unroll
  for (int c = 0; c < C8; ++c) {
    const h16x8 gg = *reinterpret_cast<const h16x8*>(g + (hl + 32 * c) * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) { gam[c][e] = (float)gg[e]; dg[c][e] = 0.f; db[c][e] = 0.f; }
  }
  for (int it = 0; it < ITERS; ++it) {
    const long row = ((long)blockIdx.x * ITERS + it) * 8 + 2 * w + half;
    if (row >= rows) break;
    const float mu = mean[row], rs = rstd[row];
    h16x8 xv[C8], dv[C8], rv[C8];
#pragma unroll
    for (int c = 0; c < C8; ++c) {
      const long off = row * D + (hl + 32 * c) * 8;
      xv[c] = *reinterpret_cast<const h16x8*>(x + off);
      dv[c] = *reinterpret_cast<const h16x8*>(dy + off);
      rv[c] = *reinterpret_cast<const h16x8*>(dres + off);
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < C8; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = ((float)xv[c][e] - mu) * rs;
        const float d = (float)dv[c][e];
        const float gd = d * gam[c][e];
        s1 += gd * xh;
        s2 += gd;
        if (ACC) { dg[c][e] += d * xh; db[c][e] += d; }
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
    s1 *= invD;
    s2 *= invD;
#pragma unroll
    for (int c = 0; c < C8; ++c) {
      h16x8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = ((float)xv[c][e] - mu) * rs;
        ov[e] = (h16)(rs * ((float)dv[c][e] * gam[c][e] - xh * s1 - s2) + (float)rv[c][e]);
      }
      *reinterpret_cast<h16x8*>(dx + row * D + (hl + 32 * c) * 8) = ov;
    }
  }
  if (!ACC) return;
#pragma unroll
  for (int c = 0; c < C8; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) { dg[c][e] += __shfl_xor(dg[c][e], 32, 64); db[c][e] += __shfl_xor(db[c][e], 32, 64); }
  if (half == 0) {
#pragma unroll
    for (int c = 0; c < C8; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) { red[w][0][(hl + 32 * c) * 8 + e] = dg[c][e]; red[w][1][(hl + 32 * c) * 8 + e] = db[c][e]; }
  }
  __syncthreads();
  float* out = part + (long)blockIdx.x * 2 * D;
  for (int i = threadIdx.x; i < 2 * D; i += 256) {
    const int which = i / D, j = i % D;
    out[i] = red[0][which][j] + red[1][which][j] + red[2][which][j] + red[3][which][j];
  }
}

int main2(h16* a, h16* b, h16* c, h16* o, long rows) {
  h16* g; float *mean, *rstd, *part;
  hipMalloc(&g, D * 2); hipMalloc(&mean, rows * 4); hipMalloc(&rstd, rows * 4); hipMalloc(&part, rows * 2 * D * 4);
  hipMemset(g, 0, D * 2); hipMemset(mean, 0, rows * 4); hipMemset(rstd, 0, rows * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = 4.0 * rows * D * 2;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 5; ++i) launch();
    hipEventRecord(e0);
    for (int i = 0; i < 50; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 50;
    printf("%-34s %7.1f us  %6.0f GB/s\n", name, us, bytes / us / 1e3);
  };
  run("V5 LN math, no acc, 1 group/blk", [&] { hipLaunchKernelGGL((v_ln<false, 1>), dim3((rows + 7) / 8), dim3(256), 0, 0, a, b, c, g, mean, rstd, o, part, rows); });
  run("V5 LN math + acc, 1 group/blk", [&] { hipLaunchKernelGGL((v_ln<true, 1>), dim3((rows + 7) / 8), dim3(256), 0, 0, a, b, c, g, mean, rstd, o, part, rows); });
  run("V5 LN math + acc, 2 groups/blk", [&] { hipLaunchKernelGGL((v_ln<true, 2>), dim3((rows + 15) / 16), dim3(256), 0, 0, a, b, c, g, mean, rstd, o, part, rows); });
  run("V5 LN math, no acc, 2 groups/blk", [&] { hipLaunchKernelGGL((v_ln<false, 2>), dim3((rows + 15) / 16), dim3(256), 0, 0, a, b, c, g, mean, rstd, o, part, rows); });
  return 0;
}

int main() {
  const long rows = 10000;
  const size_t n = rows * D;
  h16 *a, *b, *c, *o;
  hipMalloc(&a, n * 2); hipMalloc(&b, n * 2); hipMalloc(&c, n * 2); hipMalloc(&o, n * 2);
  hipMemset(a, 0, n * 2); hipMemset(b, 0, n * 2); hipMemset(c, 0, n * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = 4.0 * n * 2;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 5; ++i) launch();
    hipEventRecord(e0);
    for (int i = 0; i < 50; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 50;
    printf("%-34s %7.1f us  %6.0f GB/s\n", name, us, bytes / us / 1e3);
  };
  run("V0 half-wave copy (8 rows/blk)", [&] { hipLaunchKernelGGL(v_half<false>, dim3((rows + 7) / 8), dim3(256), 0, 0, a, b, c, o, rows); });
  run("V1 half-wave + row reductions", [&] { hipLaunchKernelGGL(v_half<true>, dim3((rows + 7) / 8), dim3(256), 0, 0, a, b, c, o, rows); });
  run("V2 wave per row (8-B lanes)", [&] { hipLaunchKernelGGL(v_wave, dim3((rows + 3) / 4), dim3(256), 0, 0, a, b, c, o, rows); });
  run("V3 half-wave, 2 rows each (16/blk)", [&] { hipLaunchKernelGGL(v_half2, dim3((rows + 15) / 16), dim3(256), 0, 0, a, b, c, o, rows); });
  main2(a, b, c, o, rows);
  hipDeviceSynchronize();
  return 0;
}
