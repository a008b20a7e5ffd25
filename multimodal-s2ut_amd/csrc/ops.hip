// Memory-bound kernels of the training step: LayerNorm fwd/bwd, column reductions (bias /
// LayerNorm parameter grads), masked attention softmax fwd/bwd with counter-RNG dropout,
// embeddings, GLU, im2col/col2im, the fusion-gate backward and small elementwise helpers.
// All HBM-bound: one wave per row for row ops, 8-byte (4 x fp16) vector accesses, fp32 math.
#include <stdlib.h>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

inline int grid_for(long n, int block, int cap = 8192) {
  long g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

MMS_DEV h16x4 ld4(const h16* p) { return *reinterpret_cast<const h16x4*>(p); }
MMS_DEV void st4(h16* p, float a, float b, float c, float d) {
  *reinterpret_cast<h16x4*>(p) = h16x4{(h16)a, (h16)b, (h16)c, (h16)d};
}

// ============================================================================ LayerNorm
template <int CPL>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const h16* __restrict__ x, const h16* __restrict__ g,
                                                     const h16* __restrict__ b, h16* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     long rows, int D, float eps, long grp, long grp_out,
                                                     float p, uint32_t thresh, uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = D >> 2;
  const h16* xr = x + row * D;
  float v[CPL][4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      h16x4 t = ld4(xr + ch * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[c][e] = (float)t[e]; s += v[c][e]; }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[c][e] = 0.f;
    }
  }
  const float mean = wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[c][e] - mean; ss += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / D + eps);
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
  // optional output layout: row r of group r / grp lands at (r / grp) * grp_out + r % grp (the
  // fusion attention's [B, Ti+1, Di] key layout); optional dropout on the fp16 result with the
  // counters of the unpadded element index (as a separate dropout pass over y would use)
  const long orow = grp ? (row / grp) * grp_out + row % grp : row;
  h16* yr = y + orow * D;
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      h16x4 gg = ld4(g + ch * 4), bb = ld4(b + ch * 4);
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[c][e] - mean) * rstd * (float)gg[e] + (float)bb[e];
      if (thresh) {
        bool k[4];
        mms_keep4(seed, offset + (uint64_t)(row * D + ch * 4), thresh, k);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = k[e] ? (float)(h16)o[e] * ds : 0.f;
      }
      st4(yr + ch * 4, o[0], o[1], o[2], o[3]);
    }
  }
}

// D % 256 == 0 (the model widths 256 / 512 / 768 / 1024): a half-wave per row, C8 16-B chunks per
// lane, two rows per wave and 8 per block -- twice the bytes per load instruction of the 4-wide
// kernel and two independent rows in flight per wave.  Same statistics / dropout counters.
MMS_DEV float half_sum(float v) { return xsum16(row16_sum(v)); }   // over each 32-lane half

template <int C8>
__global__ void __launch_bounds__(256) ln_fwd16_kernel(const h16* __restrict__ x, const h16* __restrict__ g,
                                                       const h16* __restrict__ b, h16* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       long rows, int D, float eps, long grp, long grp_out,
                                                       float p, uint32_t thresh, uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const long row = (long)blockIdx.x * 8 + (threadIdx.x >> 6) * 2 + (lane >> 5);
  if (row >= rows) return;
  const h16* xr = x + row * D;
  h16x8 xv[C8];
#pragma unroll
  for (int c = 0; c < C8; ++c) xv[c] = *reinterpret_cast<const h16x8*>(xr + (hl + 32 * c) * 8);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C8; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (float)xv[c][e];
  const float mean = half_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < C8; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = (float)xv[c][e] - mean; ss += d * d; }
  const float rstd = rsqrtf(half_sum(ss) / D + eps);
  if (hl == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
  const long orow = grp ? (row / grp) * grp_out + row % grp : row;
  h16* yr = y + orow * D;
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
  const MmsSite site = thresh ? mms_site(seed, offset, offset + (uint64_t)rows * D - 1) : MmsSite{false, 0u};
#pragma unroll
  for (int c = 0; c < C8; ++c) {
    const int col = (hl + 32 * c) * 8;
    const h16x8 gg = *reinterpret_cast<const h16x8*>(g + col), bb = *reinterpret_cast<const h16x8*>(b + col);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = ((float)xv[c][e] - mean) * rstd * (float)gg[e] + (float)bb[e];
    if (thresh) {
      bool k0[4], k1[4];
      const uint64_t c0 = offset + (uint64_t)(row * D + col);
      mms_keep4_site(site, seed, c0, thresh, k0);
      mms_keep4_site(site, seed, c0 + 4, thresh, k1);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = k0[e] ? (float)(h16)o[e] * ds : 0.f;
        o[e + 4] = k1[e] ? (float)(h16)o[e + 4] * ds : 0.f;
      }
    }
    h16x8 ov;
#pragma unroll
    for (int e = 0; e < 8; ++e) ov[e] = (h16)o[e];
    *reinterpret_cast<h16x8*>(yr + col) = ov;
  }
}

constexpr int LN_BWD_ROWS = 16;  // rows per block (4 consecutive rows per wave): ~600 blocks for 10k rows
constexpr int LN_RPW = 4;

// All loads of a wave's 4 rows (x, dy, dres) are issued before any arithmetic, so ~36 8-B loads
// per lane are in flight at once (the row-at-a-time loop was latency-bound at ~25 % of HBM BW).
template <int CPL>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const h16* __restrict__ dy, const h16* __restrict__ x,
                                                     const h16* __restrict__ g, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const h16* __restrict__ dres,
                                                     h16* __restrict__ dx, float* __restrict__ part,
                                                     long rows, int D, h16* __restrict__ dxd, float p,
                                                     uint32_t thresh, uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  __shared__ float red[4][2][CPL * 256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = D >> 2;
  const float dscale = thresh ? 1.f / (1.f - p) : 1.f;
  float dg[CPL][4], db[CPL][4], gam[CPL][4];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
#pragma unroll
    for (int e = 0; e < 4; ++e) { dg[c][e] = 0.f; db[c][e] = 0.f; gam[c][e] = 0.f; }
    if (ch < nch) {
      h16x4 gg = ld4(g + ch * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) gam[c][e] = (float)gg[e];
    }
  }
  const long rb = (long)blockIdx.x * LN_BWD_ROWS + w * LN_RPW;
  h16x4 xv[LN_RPW][CPL], dv[LN_RPW][CPL], rv[LN_RPW][CPL];
  float mu[LN_RPW], rs[LN_RPW];
  const h16x4 z4 = {(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
#pragma unroll
  for (int rr = 0; rr < LN_RPW; ++rr) {
    const long row = rb + rr;
    const bool ok = row < rows;
    mu[rr] = ok ? mean[row] : 0.f;
    rs[rr] = ok ? rstd[row] : 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      const bool v = ok && ch < nch;
      xv[rr][c] = v ? ld4(x + row * D + ch * 4) : z4;
      dv[rr][c] = v ? ld4(dy + row * D + ch * 4) : z4;
      rv[rr][c] = (v && dres && dx) ? ld4(dres + row * D + ch * 4) : z4;
    }
  }
  float s1[LN_RPW], s2[LN_RPW];
#pragma unroll
  for (int rr = 0; rr < LN_RPW; ++rr) {
    s1[rr] = 0.f;
    s2[rr] = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = ((float)xv[rr][c][e] - mu[rr]) * rs[rr];
        const float d = (float)dv[rr][c][e];
        const float gd = d * gam[c][e];
        s1[rr] += gd * xh;
        s2[rr] += gd;
        dg[c][e] += d * xh;
        db[c][e] += d;
      }
  }
  if (dx) {
#pragma unroll
    for (int rr = 0; rr < LN_RPW; ++rr) {
      s1[rr] = wave_sum(s1[rr]) / D;
      s2[rr] = wave_sum(s2[rr]) / D;
    }
#pragma unroll
    for (int rr = 0; rr < LN_RPW; ++rr) {
      const long row = rb + rr;
      if (row >= rows) break;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float xh = ((float)xv[rr][c][e] - mu[rr]) * rs[rr];
            o[e] = rs[rr] * ((float)dv[rr][c][e] * gam[c][e] - xh * s1[rr] - s2[rr]) + (float)rv[rr][c][e];
          }
          st4(dx + row * D + ch * 4, o[0], o[1], o[2], o[3]);
          if (dxd) {
            // the upstream sublayer's residual-branch dropout, replayed from its counters
            bool k[4] = {true, true, true, true};
            if (thresh) mms_keep4(seed, offset + (uint64_t)row * D + ch * 4, thresh, k);
            st4(dxd + row * D + ch * 4, k[0] ? o[0] * dscale : 0.f, k[1] ? o[1] * dscale : 0.f,
                k[2] ? o[2] * dscale : 0.f, k[3] ? o[3] * dscale : 0.f);
          }
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[w][0][(c * 64 + lane) * 4 + e] = dg[c][e];
      red[w][1][(c * 64 + lane) * 4 + e] = db[c][e];
    }
  __syncthreads();
  float* out = part + (long)blockIdx.x * 2 * D;
  for (int i = threadIdx.x; i < 2 * D; i += 256) {
    const int which = i / D, j = i % D;
    const int ch = j >> 2, e = j & 3;
    const int c = ch / 64, ln = ch % 64;
    const int idx = (c * 64 + ln) * 4 + e;
    out[i] = red[0][which][idx] + red[1][which][idx] + red[2][which][idx] + red[3][which][idx];
  }
}

// LayerNorm backward for D % 256 == 0 (the step's D = 768), one wave per row: lane l owns the
// 4-column quads l, l + 64, ... (C = D / 256 of them, 8-B accesses; every wave instruction covers a
// whole 512-B row segment).  Blocks take `iters` groups of 8 rows and fold their dgamma / dbeta
// into one partial row (reduced by colsum_parts on the side stream); wave w takes rows 2w, then
// 2w + 1 of each group.  Per lane: gamma, dgamma, dbeta (12 floats each at D = 768) and one row's
// x / dy / dres quads — 114-126 VGPRs, 4 waves per SIMD.  Measured against the half-wave layout
// (a half-wave per row, 24 columns per lane: 213 VGPRs, 2 waves per SIMD) and this kernel with two
// rows in flight per wave (181 VGPRs): 17.61-17.64 vs 17.69-17.71 / 17.71-17.73 ms per step
// (profiles/round3_v5_ln_bwd_ab.txt).
template <int C>
__global__ void __launch_bounds__(256) ln_bwd_w_kernel(const h16* __restrict__ dy, const h16* __restrict__ x,
                                                       const h16* __restrict__ g, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const h16* __restrict__ dres,
                                                       h16* __restrict__ dx, float* __restrict__ part,
                                                       long rows, int D, h16* __restrict__ dxd, float p,
                                                       uint32_t thresh, uint64_t seed, uint64_t offset,
                                                       long dgrp, long dgrp_out, float pin, uint32_t thin,
                                                       uint64_t sin, uint64_t oin, int iters) {
  if (thresh) seed = mms_step_seed(seed);
  if (thin) sin = mms_step_seed(sin);
  __shared__ __attribute__((aligned(16))) float red[4][2][C * 256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float dscale = thresh ? 1.f / (1.f - p) : 1.f;
  const float invD = 1.f / D;
  // emitted dropout: when every counter pair of the site shares one high word (always but across a
  // 2^33 boundary) one mixer per two elements with the site's constant half hoisted (mms_keep4_hi,
  // bit-identical to mms_keep4)
  const bool emit_hi = thresh && mms_same_hi(offset, offset + (uint64_t)rows * D - 1);
  const uint32_t emit_mix = emit_hi ? mms_hi_mix(seed, offset) : 0u;
  const MmsSite in_site = thin ? mms_site(sin, oin, oin + (uint64_t)rows * D - 1) : MmsSite{false, 0u};
  float gam[C][4], dg[C][4], db[C][4];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const h16x4 gg = ld4(g + (lane + 64 * c) * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { gam[c][e] = (float)gg[e]; dg[c][e] = 0.f; db[c][e] = 0.f; }
  }
  const h16x4 z4 = {(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
  // one row's operands (x, dy, dres quads, mean, rstd); iteration `it` of this wave is row
  // (block * iters + it / 2) * 8 + 2 w + it % 2
  struct RowIn {
    h16x4 xv[C], dv[C], rv[C];
    float mu, rs;
  };
  auto row_of = [&](int it) { return ((long)blockIdx.x * iters + it / 2) * 8 + (it % 2) + 2 * w; };
  auto load_row = [&](int it, RowIn& r) {
    const long row = row_of(it);
    const bool ok = it < 2 * iters && row < rows;
    r.mu = ok ? mean[row] : 0.f;
    r.rs = ok ? rstd[row] : 0.f;
    // (32-bit row arithmetic: the host guarantees rows * D < 2^31)
    const int r32 = (int)row, g32 = (int)dgrp;
    const int drow = g32 ? (r32 / g32) * (int)dgrp_out + r32 % g32 : r32;
    const h16* xr = x + (long)(r32 * D + lane * 4);
    const h16* dr = dy + (long)(drow * D + lane * 4);
    const h16* rr = dres + (long)(r32 * D + lane * 4);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      r.xv[c] = ok ? ld4(xr + 256 * c) : z4;
      r.dv[c] = ok ? ld4(dr + 256 * c) : z4;
      r.rv[c] = (ok && dres && dx) ? ld4(rr + 256 * c) : z4;
    }
  };
  // (loading the next row before this row's arithmetic -- two rows in flight, 140 VGPRs, 3 waves per
  // SIMD -- and twice the blocks (2048 row groups) both measured no faster: round-4 A/B,
  // gpurun_out r4n ln_ab, 26.2 vs 26.9 / 28.6 us isolated, step 17.24 vs 17.28 / 17.20 ms)
  RowIn cur;
#pragma unroll 1
  for (int it = 0; it < iters * 2; ++it) {
    const long row = row_of(it);
    if (row - 2 * w >= rows) break;   // (the group's first row: every wave leaves together)
    load_row(it, cur);
    const float mu = cur.mu, rs = cur.rs;
    if (thin) {
      // dy = dropout(dy_in) with the counters of the unpadded element index, rounded to fp16 as a
      // separate dropout pass would store it
      const float dsi = 1.f / (1.f - pin);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        bool kp[4];
        mms_keep4_site(in_site, sin, oin + (uint64_t)((int)row * D + (lane + 64 * c) * 4), thin, kp);
#pragma unroll
        for (int e = 0; e < 4; ++e) cur.dv[c][e] = (h16)(kp[e] ? (float)cur.dv[c][e] * dsi : 0.f);
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = ((float)cur.xv[c][e] - mu) * rs;
        const float d = (float)cur.dv[c][e];
        const float gd = d * gam[c][e];
        s1 += gd * xh;
        s2 += gd;
        dg[c][e] += d * xh;
        db[c][e] += d;
      }
    if (dx) {
      s1 = wave_sum(s1) * invD;
      s2 = wave_sum(s2) * invD;
      // re-derive x-hat and dy from the fp16 quads below instead of keeping the first pass's fp32
      // copies alive across the reductions (they would double the per-row registers)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        typedef unsigned int u32x2_ __attribute__((ext_vector_type(2)));
        u32x2_ a = __builtin_bit_cast(u32x2_, cur.xv[c]), b = __builtin_bit_cast(u32x2_, cur.dv[c]);
        asm volatile("" : "+v"(a), "+v"(b));
        cur.xv[c] = __builtin_bit_cast(h16x4, a);
        cur.dv[c] = __builtin_bit_cast(h16x4, b);
      }
      if (row < rows) {
        const int off0 = (int)row * D + lane * 4;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const int off = off0 + 256 * c;
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float xh = ((float)cur.xv[c][e] - mu) * rs;
            o[e] = rs * ((float)cur.dv[c][e] * gam[c][e] - xh * s1 - s2) + (float)cur.rv[c][e];
          }
          st4(dx + (long)off, o[0], o[1], o[2], o[3]);
          if (dxd) {
            bool kp[4] = {true, true, true, true};
            if (emit_hi) mms_keep4_hi(emit_mix, offset + (uint64_t)off, thresh, kp);
            else if (thresh) mms_keep4(seed, offset + (uint64_t)off, thresh, kp);
            st4(dxd + (long)off, kp[0] ? o[0] * dscale : 0.f, kp[1] ? o[1] * dscale : 0.f, kp[2] ? o[2] * dscale : 0.f,
                kp[3] ? o[3] * dscale : 0.f);
          }
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c)
    *reinterpret_cast<f32x4*>(&red[w][0][(lane + 64 * c) * 4]) = f32x4{dg[c][0], dg[c][1], dg[c][2], dg[c][3]};
#pragma unroll
  for (int c = 0; c < C; ++c)
    *reinterpret_cast<f32x4*>(&red[w][1][(lane + 64 * c) * 4]) = f32x4{db[c][0], db[c][1], db[c][2], db[c][3]};
  __syncthreads();
  float* out = part + (long)blockIdx.x * 2 * D;
  for (int i = threadIdx.x; i < 2 * D / 4; i += 256) {
    const int which = (4 * i) / D, j = 4 * i - which * D;
    f32x4 t = *reinterpret_cast<const f32x4*>(&red[0][which][j]);
#pragma unroll
    for (int v = 1; v < 4; ++v) t += *reinterpret_cast<const f32x4*>(&red[v][which][j]);
    *reinterpret_cast<f32x4*>(out + 4 * i) = t;
  }
}

// [nparts][ncol] fp32 -> ncol: a block owns 16 columns; its 1024 threads are 64 part slots x 16
// columns (lane l: column l & 15, slot 4w + (l >> 4)), slot j summing parts j, j + 64, ... -- 6x the
// blocks of a 64-column layout, so the L2-hot partials of a LayerNorm backward (~1000 parts x 2D)
// are read by enough waves to hide their latency.  Fixed summation order (deterministic).
__global__ void __launch_bounds__(1024) colsum_parts_kernel(const float* __restrict__ part, int nparts, int ncol,
                                                            h16* __restrict__ out, int accumulate) {
  __shared__ float red[64][17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, slot = 4 * w + (lane >> 4);
  const int c = blockIdx.x * 16 + col;
  // 16 loads in flight per thread before the first add (a 4-deep unroll left ~10 dependent L2 / HBM
  // round trips per thread, 32 us per launch in the step); the sum order is unchanged
  float s = 0.f;
  if (c < ncol) {
    for (int p0 = slot; p0 < nparts; p0 += 64 * 16) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int p = p0 + 64 * i;
        v[i] = p < nparts ? part[(long)p * ncol + c] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) s += v[i];
    }
  }
  red[slot][col] = s;
  __syncthreads();
  if (threadIdx.x < 16 && blockIdx.x * 16 + (int)threadIdx.x < ncol) {
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < 64; ++i) t += red[i][threadIdx.x];
    const int cc = blockIdx.x * 16 + threadIdx.x;
    if (accumulate) t += (float)out[cc];
    out[cc] = (h16)t;
  }
}

// column sums of an fp16 [rows][cols] matrix: grid (cols/256, splits); 4 waves stride the
// split's rows, each lane sums 4 adjacent columns (8-byte loads); LDS combine -> part[split][cols]
constexpr int COLSUM_MAX_SPLITS = 64;
__global__ void __launch_bounds__(256) colsum_f16_kernel(const h16* __restrict__ x, long rows, int cols, long ld,
                                                         float* __restrict__ part, int splits) {
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 4;
  const long per = (rows + splits - 1) / splits;
  const long r0 = (long)blockIdx.y * per, r1 = min(rows, r0 + per);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
#pragma unroll 4
    for (long r = r0 + w; r < r1; r += 4) {
      h16x4 v = ld4(x + r * ld + c);
      s += f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    }
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols) {
    const f32x4 t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    *reinterpret_cast<f32x4*>(part + (long)blockIdx.y * cols + c) = t;
  }
}

// ============================================================================ attention softmax
// One wave per score row; lane owns contiguous 4-key chunks (chunk = lane + 64*c).
MMS_DEV bool key_valid(int j, int i, int Tk, int klen, const uint8_t* km, int causal, int extra_key) {
  if (j >= Tk) return false;
  if (extra_key && j == Tk - 1) return true;
  if (j >= klen) return false;
  if (km && km[j]) return false;
  if (causal && j > i) return false;
  return true;
}

template <int CPL>
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const h16* __restrict__ S, h16* __restrict__ P,
                                                          h16* __restrict__ Pd, int Z, int H, int Tq, int Tk,
                                                          long ldS, const int* __restrict__ key_len,
                                                          const uint8_t* __restrict__ key_mask, long ld_mask,
                                                          int causal, int extra_key, float p, uint32_t thresh,
                                                          uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)Z * Tq) return;
  const int z = (int)(row / Tq), i = (int)(row % Tq);
  const int b = z / H;
  const int klen = key_len ? key_len[b] : Tk;
  const uint8_t* km = key_mask ? key_mask + (long)b * ld_mask : nullptr;
  const h16* sr = S + row * ldS;
  float v[CPL][4];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + c * 64) * 4;
    if (j0 < Tk) {
      h16x4 t = ld4(sr + j0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = j0 + e;
        v[c][e] = key_valid(j, i, Tk, klen, km, causal, extra_key) ? (float)t[e] : -INFINITY;
        mx = fmaxf(mx, v[c][e]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[c][e] = -INFINITY;
    }
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float ex = (v[c][e] == -INFINITY) ? 0.f : __expf(v[c][e] - mx);
      v[c][e] = ex;
      s += ex;
    }
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.f / s : 0.f;
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
  h16* pr = P + row * ldS;
  h16* pdr = Pd + row * ldS;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + c * 64) * 4;
    if (j0 < Tk) {
      float o[4], od[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = (j0 + e < Tk) ? v[c][e] * inv : 0.f;
        od[e] = o[e];
        if (thresh) {
          const bool keep = mms_keep(seed, offset + (uint64_t)row * Tk + (j0 + e), thresh);
          od[e] = keep ? o[e] * ds : 0.f;
        }
      }
      st4(pr + j0, o[0], o[1], o[2], o[3]);
      if (thresh) st4(pdr + j0, od[0], od[1], od[2], od[3]);
    }
  }
}

template <int CPL>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const h16* __restrict__ P, const h16* __restrict__ dPd,
                                                          h16* __restrict__ dS, int Z, int H, int Tq, int Tk,
                                                          long ldS, float p, uint32_t thresh, uint64_t seed,
                                                          uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)Z * Tq) return;
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
  float pv[CPL][4], gv[CPL][4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + c * 64) * 4;
    if (j0 < Tk) {
      h16x4 a = ld4(P + row * ldS + j0), g = ld4(dPd + row * ldS + j0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = j0 + e;
        float m = ds;
        if (thresh && j < Tk) m = mms_keep(seed, offset + (uint64_t)row * Tk + j, thresh) ? ds : 0.f;
        pv[c][e] = (j < Tk) ? (float)a[e] : 0.f;
        gv[c][e] = (j < Tk) ? (float)g[e] * m : 0.f;  // dP (undropped grad)
        s += pv[c][e] * gv[c][e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) { pv[c][e] = 0.f; gv[c][e] = 0.f; }
    }
  }
  s = wave_sum(s);
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + c * 64) * 4;
    if (j0 < Tk) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pv[c][e] * (gv[c][e] - s);
      st4(dS + row * ldS + j0, o[0], o[1], o[2], o[3]);
    }
  }
  (void)Z; (void)H;
}

// ============================================================================ elementwise
__global__ void dropout_kernel(const h16* __restrict__ x, h16* __restrict__ y, long n, float p,
                               uint32_t thresh, uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const float ds = 1.f / (1.f - p);
  const MmsSite site = mms_site(seed, offset, offset + (uint64_t)n - 1);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = (float)x[i];
    y[i] = (h16)(mms_keep_site(site, seed, offset + i, thresh) ? v * ds : 0.f);
  }
}

__global__ void dropout_mask_kernel(uint8_t* keep, long n, uint32_t thresh, uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    keep[i] = thresh ? (uint8_t)mms_keep(seed, offset + i, thresh) : 1;
}

__global__ void encoder_embed_kernel(const h16* __restrict__ h, const h16* __restrict__ pos,
                                     const int* __restrict__ len, h16* __restrict__ x, int B, int T,
                                     int D, float scale, float p, uint32_t thresh, uint64_t seed,
                                     uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const long n4 = (long)B * T * (D / 4);
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
  const MmsSite site = thresh ? mms_site(seed, offset, offset + (uint64_t)n4 * 4 - 1) : MmsSite{false, 0u};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long e0 = i * 4;
    const long bt = e0 / D;
    const int d0 = (int)(e0 % D);
    const int b = (int)(bt / T), t = (int)(bt % T);
    const int pidx = (t < len[b]) ? t + 2 : 1;
    h16x4 hv = ld4(h + e0), pv = ld4(pos + (long)pidx * D + d0);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = scale * (float)hv[e] + (float)pv[e];
      if (thresh) v = mms_keep_site(site, seed, offset + e0 + e, thresh) ? v * ds : 0.f;
      o[e] = v;
    }
    st4(x + e0, o[0], o[1], o[2], o[3]);
  }
}

__global__ void scale_dropout_bwd_kernel(const h16* __restrict__ dx, h16* __restrict__ dh, long n,
                                         float scale, float p, uint32_t thresh, uint64_t seed,
                                         uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
  const MmsSite site = thresh ? mms_site(seed, offset, offset + (uint64_t)n - 1) : MmsSite{false, 0u};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = (float)dx[i] * scale;
    if (thresh) v = mms_keep_site(site, seed, offset + i, thresh) ? v * ds : 0.f;
    dh[i] = (h16)v;
  }
}

// one wave per token: position = make_positions (cumsum of non-pad tokens up to t)
__global__ void token_embed_fwd_kernel(const int64_t* __restrict__ tok, const h16* __restrict__ E,
                                       const h16* __restrict__ pos, h16* __restrict__ x, int B, int T,
                                       int D, int pad, float scale, float p, uint32_t thresh,
                                       uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const int lane = threadIdx.x & 63;
  const long bt = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bt >= (long)B * T) return;
  const int b = (int)(bt / T), t = (int)(bt % T);
  const int64_t tk = tok[bt];
  int cnt = 0;
  for (int j = lane; j <= t; j += 64) cnt += (tok[(long)b * T + j] != pad);
  cnt = (int)wave_sum((float)cnt);
  const int pidx = (tk != pad) ? cnt + pad : pad;
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
  for (int d0 = lane * 4; d0 < D; d0 += 256) {
    h16x4 ev = ld4(E + tk * D + d0), pv = ld4(pos + (long)pidx * D + d0);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = scale * (float)ev[e] + (float)pv[e];
      if (thresh) v = mms_keep(seed, offset + bt * D + d0 + e, thresh) ? v * ds : 0.f;
      o[e] = v;
    }
    st4(x + bt * D + d0, o[0], o[1], o[2], o[3]);
  }
}

// Embedding-gradient scatter dE[v] += sum_{p: tok[p] = v} scale * dropout(dx[p]), deterministic:
// one block per vocabulary row, its 4 waves each walking a contiguous quarter of the token
// positions in order (4 x 64 token ids loaded per step, one ballot per 64) with no block barrier
// in the walk.  A lane owns 8 consecutive columns (16-B row loads; D/8 lane slots over TEB_PASS
// passes); every match row is added in ascending position order, then the 4 wave partials are
// summed in wave order through LDS — no float atomics, so the gradient is bit-reproducible.
constexpr int TEB_NT = 256, TEB_PASS = 2, TEB_UNROLL = 4;   // D <= 64 * 8 * TEB_PASS = 1024, D % 8 == 0
__global__ void __launch_bounds__(TEB_NT) token_embed_bwd_kernel(
    const int64_t* __restrict__ tok, const h16* __restrict__ dx, float* __restrict__ dE, long N, int D, int pad,
    float scale, float p, uint32_t thresh, uint64_t seed, uint64_t offset) {
  if (thresh) seed = mms_step_seed(seed);
  const int v = blockIdx.x;
  if (v == pad) return;  // nn.Embedding(padding_idx): no grad to the pad row
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ __attribute__((aligned(16))) float part[TEB_NT / 64][64 * 8 * TEB_PASS];
  const float ds = thresh ? 1.f / (1.f - p) : 1.f;
  float acc[TEB_PASS][8];
#pragma unroll
  for (int k = 0; k < TEB_PASS; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  const long q = ((N + 4 * 64 - 1) / (4 * 64)) * 64;   // positions per wave, whole 64-id chunks
  const long beg = w * q, end = min(N, beg + q);
  for (long c0 = beg; c0 < end; c0 += 64 * TEB_UNROLL) {
    uint64_t bits[TEB_UNROLL];
    int64_t t[TEB_UNROLL];
#pragma unroll
    for (int u = 0; u < TEB_UNROLL; ++u) {
      const long i = c0 + u * 64 + lane;
      t[u] = i < end ? tok[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < TEB_UNROLL; ++u) bits[u] = __ballot(t[u] == v);
#pragma unroll
    for (int u = 0; u < TEB_UNROLL; ++u) {
      uint64_t b = bits[u];
      while (b) {
        const long row = c0 + u * 64 + (__ffsll((unsigned long long)b) - 1);
        b &= b - 1;
#pragma unroll
        for (int k = 0; k < TEB_PASS; ++k) {
          const int d = (lane + 64 * k) * 8;
          if (d < D) {
            const h16x8 x8 = *reinterpret_cast<const h16x8*>(dx + row * D + d);
            bool kp[8] = {true, true, true, true, true, true, true, true};
            if (thresh) {
              bool k0[4], k1[4];
              mms_keep4(seed, offset + (uint64_t)(row * D + d), thresh, k0);
              mms_keep4(seed, offset + (uint64_t)(row * D + d) + 4, thresh, k1);
#pragma unroll
              for (int e = 0; e < 4; ++e) { kp[e] = k0[e]; kp[e + 4] = k1[e]; }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float xv = (float)x8[e] * scale;
              acc[k][e] += thresh ? (kp[e] ? xv * ds : 0.f) : xv;
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < TEB_PASS; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) part[w][(lane + 64 * k) * 8 + e] = acc[k][e];
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += TEB_NT)
    dE[(long)v * D + d] += ((part[0][d] + part[1][d]) + part[2][d]) + part[3][d];
}

__global__ void add_f32_to_f16_kernel(const h16* __restrict__ a, const float* __restrict__ b,
                                      h16* __restrict__ out, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (h16)((float)a[i] + b[i]);
}

__global__ void add_f16_kernel(const h16* __restrict__ a, const h16* __restrict__ b,
                               h16* __restrict__ out, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (h16)((float)a[i] + (float)b[i]);
}

MMS_DEV float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ void glu_fwd_kernel(const h16* __restrict__ x, h16* __restrict__ y, long rows, int C) {
  const long n4 = rows * (C / 4);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long r = i / (C / 4);
    const int c = (int)(i % (C / 4)) * 4;
    h16x4 a = ld4(x + r * 2 * C + c), g = ld4(x + r * 2 * C + C + c);
    st4(y + r * C + c, (float)a[0] * sigm((float)g[0]), (float)a[1] * sigm((float)g[1]),
        (float)a[2] * sigm((float)g[2]), (float)a[3] * sigm((float)g[3]));
  }
}

__global__ void glu_bwd_kernel(const h16* __restrict__ x, const h16* __restrict__ dy,
                               h16* __restrict__ dx, long rows, int C) {
  const long n4 = rows * (C / 4);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long r = i / (C / 4);
    const int c = (int)(i % (C / 4)) * 4;
    h16x4 a = ld4(x + r * 2 * C + c), g = ld4(x + r * 2 * C + C + c), d = ld4(dy + r * C + c);
    float da[4], dg[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float s = sigm((float)g[e]);
      da[e] = (float)d[e] * s;
      dg[e] = (float)d[e] * (float)a[e] * s * (1.f - s);
    }
    st4(dx + r * 2 * C + c, da[0], da[1], da[2], da[3]);
    st4(dx + r * 2 * C + C + c, dg[0], dg[1], dg[2], dg[3]);
  }
}

// col[(b,t)][c*k + kk] = x[b][t*stride - pad + kk][c]
// col rows are ldcol >= C*k wide; columns [C*k, ldcol) are written as zeros (a K padded to whole
// 64-wide k-tiles for the LDS-DMA GEMM)
__global__ void im2col_kernel(const h16* __restrict__ x, h16* __restrict__ col, int B, int Tin,
                              int Tout, int C, int k, int stride, int pad, int ldcol) {
  const int W = C * k;
  const long n = (long)B * Tout * ldcol;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long bt = i / ldcol;
    const int rem = (int)(i % ldcol);
    const int c = rem / k, kk = rem % k;
    const int b = (int)(bt / Tout), t = (int)(bt % Tout);
    const int ti = t * stride - pad + kk;
    col[i] = (rem < W && ti >= 0 && ti < Tin) ? x[((long)b * Tin + ti) * C + c] : (h16)0.f;
  }
}

// im2col with 8 consecutive columns of one row per thread (one 16-B store) and 32-bit index math
// (the generic kernel's 64-bit div/mod per element dominated it): ldcol % 8 == 0, col 16-B aligned,
// B*Tout*ldcol < 2^31.  The x gathers of a row's 8 columns hit at most 2 channel positions x k taps.
__global__ void im2col8_kernel(const h16* __restrict__ x, h16* __restrict__ col, int rows, int Tin, int Tout,
                               int C, int k, int stride, int pad, int ldcol) {
  const int W = C * k, n8 = ldcol >> 3, total = rows * n8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int bt = i / n8, r8 = (i - bt * n8) << 3;
    const int b = bt / Tout, t = bt - b * Tout;
    const int t0 = t * stride - pad;
    const h16* xb = x + (long)b * Tin * C;
    int c = r8 / k, kk = r8 - c * k;
    h16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ti = t0 + kk;
      v[e] = (r8 + e < W && ti >= 0 && ti < Tin) ? xb[ti * C + c] : (h16)0.f;
      if (++kk == k) { kk = 0; ++c; }
    }
    *reinterpret_cast<h16x8*>(col + (long)bt * ldcol + r8) = v;
  }
}

// col2im with 4 consecutive channels per thread (one 8-B store), 32-bit index math: C % 4 == 0,
// B*Tin*C < 2^31.  Same summation order as col2im_kernel (taps kk ascending, fp32).
__global__ void col2im4_kernel(const h16* __restrict__ dcol, h16* __restrict__ dx, int rows_in, int Tin,
                               int Tout, int C, int k, int stride, int pad) {
  const int C4 = C >> 2, total = rows_in * C4, W = C * k;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int bt = i / C4, c = (i - bt * C4) << 2;
    const int b = bt / Tin, ti = bt - b * Tin;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int kk = 0; kk < k; ++kk) {
      const int num = ti + pad - kk;
      if (num < 0 || num % stride) continue;
      const int t = num / stride;
      if (t >= Tout) continue;
      const h16* src = dcol + (long)(b * Tout + t) * W + c * k + kk;
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += (float)src[e * k];
    }
    *reinterpret_cast<h16x4*>(dx + (long)bt * C + c) = h16x4{(h16)s[0], (h16)s[1], (h16)s[2], (h16)s[3]};
  }
}

__global__ void col2im_kernel(const h16* __restrict__ dcol, h16* __restrict__ dx, int B, int Tin,
                              int Tout, int C, int k, int stride, int pad) {
  const long n = (long)B * Tin * C;
  const long W = (long)C * k;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long bt = i / C;
    const int b = (int)(bt / Tin), ti = (int)(bt % Tin);
    float s = 0.f;
    for (int kk = 0; kk < k; ++kk) {
      const int num = ti + pad - kk;
      if (num < 0 || num % stride) continue;
      const int t = num / stride;
      if (t >= Tout) continue;
      s += (float)dcol[((long)b * Tout + t) * W + (long)c * k + kk];
    }
    dx[i] = (h16)s;
  }
}

__global__ void gate_bwd_kernel(const h16* __restrict__ dres, const h16* __restrict__ merge,
                                const h16* __restrict__ g, h16* __restrict__ dpre,
                                h16* __restrict__ dmerge, long rows, int D) {
  const long n4 = rows * (D / 4);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long r = i / (D / 4);
    const int c = (int)(i % (D / 4)) * 4;
    h16x4 dr = ld4(dres + r * D + c), o = ld4(merge + r * 2 * D + c), t = ld4(merge + r * 2 * D + D + c),
          gv = ld4(g + r * D + c);
    float dp[4], dmo[4], dmt[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gg = (float)gv[e], d = (float)dr[e];
      dp[e] = d * ((float)o[e] - (float)t[e]) * gg * (1.f - gg);
      dmo[e] = d * gg;
      dmt[e] = d * (1.f - gg);
    }
    st4(dpre + r * D + c, dp[0], dp[1], dp[2], dp[3]);
    st4(dmerge + r * 2 * D + c, dmo[0], dmo[1], dmo[2], dmo[3]);
    st4(dmerge + r * 2 * D + D + c, dmt[0], dmt[1], dmt[2], dmt[3]);
  }
}

// dst row r = [src row r (cols) | zcols zeros]; VEC: 8 halves per item (every stride, count and
// base 8-aligned), else one
template <int VEC>
__global__ void copy2d_kernel(const h16* __restrict__ src, long lds, h16* __restrict__ dst, long ldd,
                              long rows, int cols, int zcols) {
  const int w = (cols + zcols) / VEC, cv = cols / VEC;
  const long n = rows * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / w;
    const int c = (int)(i % w);
    if (VEC == 8) {
      s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (c < cv) v = *reinterpret_cast<const s16x8*>(src + r * lds + 8 * c);
      *reinterpret_cast<s16x8*>(dst + r * ldd + 8 * c) = v;
    } else {
      dst[r * ldd + c] = c < cv ? src[r * lds + c] : (h16)0.f;
    }
  }
}

template <typename F>
int pick_cpl(int chunks_per_row, F&& f) {
  const int cpl = (chunks_per_row + 63) / 64;
  if (cpl <= 1) return f(std::integral_constant<int, 1>{});
  if (cpl <= 2) return f(std::integral_constant<int, 2>{});
  if (cpl <= 3) return f(std::integral_constant<int, 3>{});
  if (cpl <= 4) return f(std::integral_constant<int, 4>{});
  if (cpl <= 8) return f(std::integral_constant<int, 8>{});
  if (cpl <= 16) return f(std::integral_constant<int, 16>{});
  mms::set_error("row too long (%d chunks)", chunks_per_row);
  return 1;
}

}  // namespace

// the half-wave LayerNorm forward: D a multiple of 256 (<= 1024), 16-B aligned rows and operands
static bool ln_fwd16_ok(const h16* x, const h16* g, const h16* b, const h16* y, int D) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return D % 256 == 0 && D <= 1024 && al(x) && al(g) && al(b) && al(y);
}

static int ln_fwd16_launch(const h16* x, const h16* g, const h16* b, h16* y, float* mean, float* rstd,
                           int64_t rows, int D, float eps, int64_t grp, int64_t grp_out, float p, uint32_t th,
                           uint64_t seed, uint64_t offset, hipStream_t s) {
  const dim3 grid((unsigned)((rows + 7) / 8)), block(256);
  switch (D / 256) {
#define CASE(C) case C: hipLaunchKernelGGL((ln_fwd16_kernel<C>), grid, block, 0, s, x, g, b, y, mean, rstd, \
                                           (long)rows, D, eps, (long)grp, (long)grp_out, p, th, seed, offset); break;
    CASE(1) CASE(2) CASE(3) CASE(4)
#undef CASE
    default: mms::set_error("layernorm_fwd16: D=%d", D); return 1;
  }
  return mms::check_launch("layernorm_fwd16");
}

// ============================================================================ C-ABI
extern "C" int mms2ut_layernorm_fwd(const h16* x, const h16* gamma, const h16* beta, h16* y,
                                    float* mean, float* rstd, int64_t rows, int D, float eps,
                                    hipStream_t s) {
  MMS_REQUIRE(D % 4 == 0, "layernorm: D must be a multiple of 4");
  if (rows == 0) return 0;
  if (ln_fwd16_ok(x, gamma, beta, y, D))
    return ln_fwd16_launch(x, gamma, beta, y, mean, rstd, rows, D, eps, 0, 0, 0.f, 0u, 0, 0, s);
  return pick_cpl(D / 4, [&](auto C) {
    hipLaunchKernelGGL((ln_fwd_kernel<decltype(C)::value>), dim3((rows + 3) / 4), dim3(256), 0, s,
                       x, gamma, beta, y, mean, rstd, (long)rows, D, eps, 0L, 0L, 0.f, 0u, (uint64_t)0,
                       (uint64_t)0);
    return mms::check_launch("layernorm_fwd");
  });
}

extern "C" int mms2ut_layernorm_fwd_ex(const h16* x, const h16* gamma, const h16* beta, h16* y,
                                       float* mean, float* rstd, int64_t rows, int D, float eps,
                                       int64_t grp, int64_t grp_out, float p, uint64_t seed,
                                       uint64_t offset, hipStream_t s) {
  MMS_REQUIRE(D % 4 == 0, "layernorm_fwd_ex: D must be a multiple of 4");
  MMS_REQUIRE(grp >= 0 && (grp == 0 || grp_out >= grp), "layernorm_fwd_ex: need grp_out >= grp");
  MMS_REQUIRE(p < 1.f, "layernorm_fwd_ex: p must be < 1");
  if (rows == 0) return 0;
  const uint32_t th = mms_drop_thresh(p);
  if (ln_fwd16_ok(x, gamma, beta, y, D))
    return ln_fwd16_launch(x, gamma, beta, y, mean, rstd, rows, D, eps, grp, grp_out, p, th, seed, offset, s);
  return pick_cpl(D / 4, [&](auto C) {
    hipLaunchKernelGGL((ln_fwd_kernel<decltype(C)::value>), dim3((rows + 3) / 4), dim3(256), 0, s,
                       x, gamma, beta, y, mean, rstd, (long)rows, D, eps, (long)grp, (long)grp_out, p, th,
                       seed, offset);
    return mms::check_launch("layernorm_fwd_ex");
  });
}

static bool ln16_path(int D) { return D % 256 == 0 && D <= 1024; }

extern "C" int mms2ut_layernorm_bwd_parts(int64_t rows) {
  return (int)((rows + LN_BWD_ROWS - 1) / LN_BWD_ROWS);
}

// groups of 8 rows per ln_bwd_w block: enough blocks to fill the chip (1024), each folding its
// groups' dgamma / dbeta into one partial row — the partials (rows / 8 x 6 KB at D = 768 before
// the folding) are what colsum_parts reads back on the side stream
static int ln16_iters(int64_t rows) {
  constexpr long target = 1024;
  const long groups = (rows + 7) / 8;
  const long it = (groups + target - 1) / target;
  return (int)(it > 1 ? it : 1);
}

extern "C" int mms2ut_layernorm_bwd_nparts(int64_t rows, int D) {
  if (!ln16_path(D)) return (int)((rows + LN_BWD_ROWS - 1) / LN_BWD_ROWS);
  const long rpb = 8L * ln16_iters(rows);
  return (int)((rows + rpb - 1) / rpb);
}

extern "C" int mms2ut_layernorm_bwd(const h16* dy, const h16* x, const h16* gamma, const float* mean,
                                    const float* rstd, const h16* dres, h16* dx, float* part,
                                    int64_t rows, int D, h16* dxd, float p, uint64_t seed,
                                    uint64_t offset, hipStream_t s) {
  MMS_REQUIRE(!dxd || dx, "layernorm_bwd: dxd needs dx");
  MMS_REQUIRE(p < 1.f, "layernorm_bwd: p must be < 1");
  const uint32_t thresh = mms_drop_thresh(p);
  MMS_REQUIRE(D % 4 == 0 && D <= 1024, "layernorm_bwd: D must be a multiple of 4 and <= 1024");
  if (rows == 0) return 0;
  const int nb = mms2ut_layernorm_bwd_nparts(rows, D);
  if (ln16_path(D)) {
    MMS_REQUIRE(rows * D < (1LL << 31), "layernorm_bwd: rows * D must be < 2^31 (32-bit row offsets)");
#define CASE(C) case C: hipLaunchKernelGGL((ln_bwd_w_kernel<C>), dim3(nb), dim3(256), 0, s, dy, x, gamma, mean, \
                                           rstd, dres, dx, part, (long)rows, D, dxd, p, thresh, seed, offset, 0L, \
                                           0L, 0.f, 0u, (uint64_t)0, (uint64_t)0, ln16_iters(rows)); break;
    switch (D / 256) { CASE(1) CASE(2) CASE(3) CASE(4) }
#undef CASE
    return mms::check_launch("layernorm_bwd_w");
  }
  return pick_cpl(D / 4, [&](auto C) {
    constexpr int CPL = decltype(C)::value;
    if constexpr (CPL <= 4) {
      hipLaunchKernelGGL((ln_bwd_kernel<CPL>), dim3(nb), dim3(256), 0, s, dy, x, gamma, mean, rstd,
                         dres, dx, part, (long)rows, D, dxd, p, thresh, seed, offset);
      return mms::check_launch("layernorm_bwd");
    } else {
      mms::set_error("layernorm_bwd: D too large");
      return 1;
    }
  });
}

extern "C" int mms2ut_layernorm_bwd_ex(const h16* dy, const h16* x, const h16* gamma, const float* mean,
                                       const float* rstd, const h16* dres, h16* dx, float* part,
                                       int64_t rows, int D, h16* dxd, float p, uint64_t seed, uint64_t offset,
                                       int64_t dy_grp, int64_t dy_grp_out, float dy_p, uint64_t dy_seed,
                                       uint64_t dy_offset, hipStream_t s) {
  MMS_REQUIRE(!dxd || dx, "layernorm_bwd_ex: dxd needs dx");
  MMS_REQUIRE(p < 1.f && dy_p < 1.f, "layernorm_bwd_ex: p must be < 1");
  MMS_REQUIRE(D % 256 == 0 && D <= 1024, "layernorm_bwd_ex: D must be a multiple of 256 and <= 1024");
  MMS_REQUIRE(dy_grp >= 0 && (dy_grp == 0 || dy_grp_out >= dy_grp), "layernorm_bwd_ex: need dy_grp_out >= dy_grp");
  if (rows == 0) return 0;
  const int nb = mms2ut_layernorm_bwd_nparts(rows, D);
  const uint32_t thresh = mms_drop_thresh(p), thin = mms_drop_thresh(dy_p);
  MMS_REQUIRE(rows * D < (1LL << 31) && (dy_grp == 0 || (rows / dy_grp + 1) * dy_grp_out * D < (1LL << 31)),
              "layernorm_bwd_ex: row offsets must fit 32 bits");
#define CASE(C) case C: hipLaunchKernelGGL((ln_bwd_w_kernel<C>), dim3(nb), dim3(256), 0, s, dy, x, gamma, mean, \
                                           rstd, dres, dx, part, (long)rows, D, dxd, p, thresh, seed, offset, \
                                           (long)dy_grp, (long)dy_grp_out, dy_p, thin, dy_seed, dy_offset, \
                                           ln16_iters(rows)); break;
  switch (D / 256) { CASE(1) CASE(2) CASE(3) CASE(4) }
#undef CASE
  return mms::check_launch("layernorm_bwd_ex");
}

extern "C" int mms2ut_colsum_parts(const float* part, int nparts, int ncol, h16* out, int accumulate,
                                   hipStream_t s) {
  if (ncol == 0) return 0;
  hipLaunchKernelGGL(colsum_parts_kernel, dim3((ncol + 15) / 16), dim3(1024), 0, s, part, nparts,
                     ncol, out, accumulate);
  return mms::check_launch("colsum_parts");
}

extern "C" int mms2ut_colsum_nparts(int64_t rows) {
  long sp = (rows + 63) / 64;
  if (sp > COLSUM_MAX_SPLITS) sp = COLSUM_MAX_SPLITS;
  return sp < 1 ? 1 : (int)sp;
}

extern "C" int mms2ut_colsum_f16(const h16* x, int64_t rows, int cols, int64_t ld, float* part,
                                 int nparts, hipStream_t s) {
  MMS_REQUIRE(cols % 4 == 0 && ld % 4 == 0, "colsum_f16: cols/ld must be multiples of 4");
  MMS_REQUIRE(nparts == mms2ut_colsum_nparts(rows), "colsum_f16: nparts mismatch");
  if (rows == 0) return 0;
  dim3 grid((cols / 4 + 63) / 64, nparts);
  hipLaunchKernelGGL(colsum_f16_kernel, grid, dim3(256), 0, s, x, (long)rows, cols, (long)ld, part, nparts);
  return mms::check_launch("colsum_f16");
}

extern "C" int mms2ut_attn_softmax_fwd(const h16* S, h16* P, h16* Pd, int Z, int H, int Tq, int Tk,
                                       int64_t ldS, const int32_t* key_len, const uint8_t* key_mask,
                                       int64_t ld_mask, int causal, int extra_key,
                                       float p, uint64_t seed, uint64_t offset, hipStream_t s) {
  MMS_REQUIRE(ldS % 4 == 0 && ldS >= Tk, "softmax: ldS must be a multiple of 4 and >= Tk");
  MMS_REQUIRE(p < 1.f, "softmax: p must be < 1");
  const long rows = (long)Z * Tq;
  if (rows == 0) return 0;
  const uint32_t th = mms_drop_thresh(p);
  return pick_cpl((Tk + 3) / 4, [&](auto C) {
    hipLaunchKernelGGL((softmax_fwd_kernel<decltype(C)::value>), dim3((rows + 3) / 4), dim3(256), 0, s,
                       S, P, Pd, Z, H, Tq, Tk, (long)ldS, key_len, key_mask, (long)ld_mask, causal,
                       extra_key, p, th, seed, offset);
    return mms::check_launch("attn_softmax_fwd");
  });
}

extern "C" int mms2ut_attn_softmax_bwd(const h16* P, const h16* dPd, h16* dS, int Z, int H, int Tq,
                                       int Tk, int64_t ldS, const int32_t* key_len, int causal,
                                       int extra_key, float p, uint64_t seed, uint64_t offset,
                                       hipStream_t s) {
  MMS_REQUIRE(ldS % 4 == 0 && ldS >= Tk, "softmax_bwd: ldS must be a multiple of 4 and >= Tk");
  const long rows = (long)Z * Tq;
  if (rows == 0) return 0;
  const uint32_t th = mms_drop_thresh(p);
  (void)key_len; (void)causal; (void)extra_key;  // masked entries have P == 0 -> dS == 0
  return pick_cpl((Tk + 3) / 4, [&](auto C) {
    hipLaunchKernelGGL((softmax_bwd_kernel<decltype(C)::value>), dim3((rows + 3) / 4), dim3(256), 0, s,
                       P, dPd, dS, Z, H, Tq, Tk, (long)ldS, p, th, seed, offset);
    return mms::check_launch("attn_softmax_bwd");
  });
}

extern "C" int mms2ut_dropout_fwd(const h16* x, h16* y, int64_t n, float p, uint64_t seed,
                                  uint64_t offset, hipStream_t s) {
  MMS_REQUIRE(p < 1.f, "dropout: p must be < 1");
  if (n == 0) return 0;
  const uint32_t th = mms_drop_thresh(p);
  if (!th) {
    if (x != y) return hipMemcpyAsync(y, x, n * 2, hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : 1;
    return 0;
  }
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, y, (long)n, p, th, seed, offset);
  return mms::check_launch("dropout_fwd");
}

extern "C" int mms2ut_dropout_mask(uint8_t* keep, int64_t n, float p, uint64_t seed, uint64_t offset,
                                   hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, keep, (long)n,
                     mms_drop_thresh(p), seed, offset);
  return mms::check_launch("dropout_mask");
}

extern "C" int mms2ut_encoder_embed_fwd(const h16* h, const h16* pos, const int32_t* len, h16* x, int B,
                                        int T, int D, float scale, float p, uint64_t seed,
                                        uint64_t offset, hipStream_t s) {
  MMS_REQUIRE(D % 4 == 0, "encoder_embed: D must be a multiple of 4");
  const long n4 = (long)B * T * (D / 4);
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(encoder_embed_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, h, pos, len, x, B,
                     T, D, scale, p, mms_drop_thresh(p), seed, offset);
  return mms::check_launch("encoder_embed_fwd");
}

extern "C" int mms2ut_scale_dropout_bwd(const h16* dx, h16* dh, int64_t n, float scale, float p,
                                        uint64_t seed, uint64_t offset, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(scale_dropout_bwd_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, dx, dh, (long)n,
                     scale, p, mms_drop_thresh(p), seed, offset);
  return mms::check_launch("scale_dropout_bwd");
}

extern "C" int mms2ut_token_embed_fwd(const int64_t* tok, const h16* E, const h16* pos, h16* x, int B,
                                      int T, int D, int pad_idx, float scale, float p, uint64_t seed,
                                      uint64_t offset, hipStream_t s) {
  MMS_REQUIRE(D % 4 == 0, "token_embed: D must be a multiple of 4");
  const long n = (long)B * T;
  if (n == 0) return 0;
  hipLaunchKernelGGL(token_embed_fwd_kernel, dim3((n + 3) / 4), dim3(256), 0, s, tok, E, pos, x, B, T,
                     D, pad_idx, scale, p, mms_drop_thresh(p), seed, offset);
  return mms::check_launch("token_embed_fwd");
}

extern "C" int mms2ut_token_embed_bwd(const int64_t* tok, const h16* dx, float* dE32, int B, int T,
                                      int D, int V, int pad_idx, float scale, float p, uint64_t seed,
                                      uint64_t offset, hipStream_t s) {
  MMS_REQUIRE(D > 0 && D <= 64 * 8 * TEB_PASS && D % 8 == 0 && V > 0,
              "token_embed_bwd: D=%d (max %d, a multiple of 8) V=%d", D, 64 * 8 * TEB_PASS, V);
  MMS_REQUIRE(((uintptr_t)dx & 15) == 0, "token_embed_bwd: dx must be 16-B aligned");
  const long n = (long)B * T;
  if (n == 0) return 0;
  hipLaunchKernelGGL(token_embed_bwd_kernel, dim3(V), dim3(TEB_NT), 0, s, tok, dx, dE32, n, D,
                     pad_idx, scale, p, mms_drop_thresh(p), seed, offset);
  return mms::check_launch("token_embed_bwd");
}

extern "C" int mms2ut_add_f32_to_f16(const h16* a, const float* b, h16* out, int64_t n, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(add_f32_to_f16_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, a, b, out, (long)n);
  return mms::check_launch("add_f32_to_f16");
}

extern "C" int mms2ut_add_f16(const h16* a, const h16* b, h16* out, int64_t n, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(add_f16_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, a, b, out, (long)n);
  return mms::check_launch("add_f16");
}

extern "C" int mms2ut_glu_fwd(const h16* x, h16* y, int64_t rows, int C, hipStream_t s) {
  MMS_REQUIRE(C % 4 == 0, "glu: C must be a multiple of 4");
  const long n4 = (long)rows * (C / 4);
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(glu_fwd_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, x, y, (long)rows, C);
  return mms::check_launch("glu_fwd");
}

extern "C" int mms2ut_glu_bwd(const h16* x, const h16* dy, h16* dx, int64_t rows, int C, hipStream_t s) {
  MMS_REQUIRE(C % 4 == 0, "glu_bwd: C must be a multiple of 4");
  const long n4 = (long)rows * (C / 4);
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(glu_bwd_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, x, dy, dx, (long)rows, C);
  return mms::check_launch("glu_bwd");
}

extern "C" int mms2ut_im2col_ld(const h16* x, h16* col, int B, int Tin, int Tout, int C, int k, int stride,
                                int pad, int ldcol, hipStream_t s) {
  MMS_REQUIRE(ldcol >= C * k, "im2col: ldcol < C*k");
  const long n = (long)B * Tout * ldcol;
  if (n == 0) return 0;
  if (ldcol % 8 == 0 && ((uintptr_t)col & 15) == 0 && n < (1L << 31)) {
    hipLaunchKernelGGL(im2col8_kernel, dim3(grid_for(n / 8, 256)), dim3(256), 0, s, x, col, B * Tout, Tin, Tout,
                       C, k, stride, pad, ldcol);
    return mms::check_launch("im2col");
  }
  hipLaunchKernelGGL(im2col_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, col, B, Tin, Tout, C, k,
                     stride, pad, ldcol);
  return mms::check_launch("im2col");
}

extern "C" int mms2ut_im2col(const h16* x, h16* col, int B, int Tin, int Tout, int C, int k, int stride,
                             int pad, hipStream_t s) {
  return mms2ut_im2col_ld(x, col, B, Tin, Tout, C, k, stride, pad, C * k, s);
}

extern "C" int mms2ut_col2im(const h16* dcol, h16* dx, int B, int Tin, int Tout, int C, int k, int stride,
                             int pad, hipStream_t s) {
  const long n = (long)B * Tin * C;
  if (n == 0) return 0;
  if (C % 4 == 0 && ((uintptr_t)dx & 7) == 0 && n < (1L << 31) && (long)B * Tout * C * k < (1L << 31)) {
    hipLaunchKernelGGL(col2im4_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, s, dcol, dx, B * Tin, Tin, Tout,
                       C, k, stride, pad);
    return mms::check_launch("col2im");
  }
  hipLaunchKernelGGL(col2im_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, dcol, dx, B, Tin, Tout, C, k,
                     stride, pad);
  return mms::check_launch("col2im");
}

extern "C" int mms2ut_gate_bwd(const h16* dres, const h16* merge, const h16* g, h16* dpre, h16* dmerge,
                               int64_t rows, int D, hipStream_t s) {
  MMS_REQUIRE(D % 4 == 0, "gate_bwd: D must be a multiple of 4");
  const long n4 = (long)rows * (D / 4);
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(gate_bwd_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, dres, merge, g, dpre,
                     dmerge, (long)rows, D);
  return mms::check_launch("gate_bwd");
}

extern "C" int mms2ut_copy2d_pad(const h16* src, int64_t lds, h16* dst, int64_t ldd, int64_t rows, int cols,
                                 int zcols, hipStream_t s) {
  MMS_REQUIRE(rows >= 0 && cols >= 0 && zcols >= 0 && (cols == 0 || src) && dst, "copy2d_pad: bad arguments");
  MMS_REQUIRE(rows <= 1 || ldd >= cols + zcols, "copy2d_pad: dst rows overlap");
  const long n = (long)rows * (cols + zcols);
  if (n == 0) return 0;
  const bool v8 = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0 && (lds | ldd | cols | zcols) % 8 == 0;
  if (v8) {
    hipLaunchKernelGGL((copy2d_kernel<8>), dim3(grid_for(n / 8, 256)), dim3(256), 0, s, src, (long)lds, dst,
                       (long)ldd, (long)rows, cols, zcols);
  } else {
    hipLaunchKernelGGL((copy2d_kernel<1>), dim3(grid_for(n, 256)), dim3(256), 0, s, src, (long)lds, dst,
                       (long)ldd, (long)rows, cols, zcols);
  }
  return mms::check_launch("copy2d");
}

extern "C" int mms2ut_copy2d(const h16* src, int64_t lds, h16* dst, int64_t ldd, int64_t rows, int cols,
                             hipStream_t s) {
  return mms2ut_copy2d_pad(src, lds, dst, ldd, rows, cols, 0, s);
}

namespace mms {
int bind_step_seed_ops(const uint64_t* d) { return mms_bind_step_seed_tu(d); }
}  // namespace mms
