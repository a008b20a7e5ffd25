// Persistent NT GEMM with deferred C stores (gfx950): C[M, N] = epilogue(A[M, K] . B[N, K]^T), both
// operands K-contiguous — the step's forward projections and, through the W^T images, its dgrads.
//
// Why: with one tile per block every tile of a round ends its k-loop together, so all 256 CUs
// write C at the same moment (a ~5 TB/s burst the matrix cores wait behind) and every tile pays
// its prologue load latency with an empty pipe.  Here 2 blocks per CU walk a static sequence of
// tiles; after tile i's k-loop a block
//   1. DMAs tile i+1's first k-stage into the idle half of its LDS ring,
//   2. runs tile i's epilogue straight from the accumulators (MFMA layout, no LDS staging: each
//      fragment's bias / residual / dropout math on the lane's 4 columns, then v_permlane16_swap
//      pairs fragments j, j+1 so a lane holds 8 consecutive columns = one 16-B store), and
//   3. keeps the packed fp16 results in registers and stores them a few per k-step during tile
//      i+1's k-loop, behind that step's DMA (the step's counted vmcnt leaves them in flight),
// so C leaves the CU spread over the next tile's k-loop instead of in one chip-wide burst.
//
// The k-loop is gemm_tall_kernel's (32 FRT x 128 tiles, 4 waves of 16 FRT x 64, 2-stage LDS-DMA
// ring, XOR-swizzled images, mfma_f32_16x16x32_f16 with (B, A) swapped), the epilogue arithmetic is
// staged_epilogue's element for element and the dropout keep bits the same hash of the same
// counters: results are bit-identical to gemm_dma_kernel.
#pragma once
#include "lab_gemm_wide.h"   // wait_vm_n

namespace mmsp {
namespace {

typedef unsigned int pu32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int pu32x4 __attribute__((ext_vector_type(4)));

template <int EPI>
constexpr bool pt_supported() {
  return EPI == MMS_EPI_F16 || EPI == MMS_EPI_RELU_DROP || EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_RELU_DROP_BWD;
}
template <int EPI>
constexpr bool pt_aux() {
  return EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_RELU_DROP_BWD;
}

// tile-uniform dropout state: the fast path (every counter of the tile shares its pair index's high
// word; even offset and row stride) mixes one 32-bit word per element pair
struct PtDrop {
  bool fast;
  uint32_t hmix, pbase;
};

// staged_epilogue's arithmetic on one fragment (lane's 4 columns n0..n0+3 of row m) -> 4 fp16
template <int EPI>
MMS_DEV pu32x2 pt_frag(const GemmP& P, const f32x4& v, const float (&bv)[4], const h16x4& ax, const PtDrop& D,
                       uint32_t pair0, int m, int n0, float dscale) {
  float x[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] = v[e] * P.alpha + bv[e];
  bool keep[4] = {true, true, true, true};
  if (epi_drops<EPI>() && P.thresh) {
    if (D.fast) {
      const uint32_t h0 = mms_mix32(pair0 ^ D.hmix), h1 = mms_mix32((pair0 + 1) ^ D.hmix);
      keep[0] = (h0 & 0xffffU) >= P.thresh;
      keep[1] = (h0 >> 16) >= P.thresh;
      keep[2] = (h1 & 0xffffU) >= P.thresh;
      keep[3] = (h1 >> 16) >= P.thresh;
    } else {
      mms_keep4(P.seed, P.offset + (uint64_t)m * P.ld_rng + n0, P.thresh, keep);
    }
  }
  h16x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float r;
    if (EPI == MMS_EPI_RELU_DROP) r = keep[e] ? fmaxf(x[e], 0.f) * dscale : 0.f;
    else if (EPI == MMS_EPI_DROP_RESID) r = (float)ax[e] + (keep[e] ? x[e] * dscale : 0.f);
    else if (EPI == MMS_EPI_RELU_DROP_BWD) r = (float)ax[e] > 0.f ? x[e] * dscale : 0.f;
    else r = x[e];
    o[e] = (h16)r;
  }
  return __builtin_bit_cast(pu32x2, o);
}

// DEFER: stores of tile i go out during tile i+1's k-loop (else right after the math)
template <int EPI, int FRT, bool DEFER>
__global__ void __launch_bounds__(NT, 2) gemm_persist_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  constexpr int BMT = 32 * FRT, TILE_T = BMT * 64 * 2, STAGE = TILE_T + TILE_BYTES;
  constexpr int NST = 2 * FRT;   // 16-B stores per lane per tile (fragment pairs)
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int q = lane >> 4, r16 = lane & 15;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.A, (short)0, (int)(((long)(P.M - 1) * P.lda + P.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.B, (short)0, (int)(((long)(P.N - 1) * P.ldb + P.K) * 2), 0x00020000);
  const int nk = P.K / BK;   // host: K % 64 == 0, K > 0
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  const bool drop_ok = ((P.offset & 1) == 0) && ((P.ld_rng & 1) == 0);
  h16* C = reinterpret_cast<h16*>(P.C);

  auto stage_a = [&](int s) { return smem + s * STAGE; };
  auto stage_b = [&](int s) { return smem + s * STAGE + TILE_T; };
  auto coords = [&](int lin, int& bm, int& bn) {
    int z, tm, tn;
    tile_coords(lin, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
    bm = tm * BMT;
    bn = tn * BN;
  };
  auto dma_stage = [&](int s, int bm, int bn, int k0) {
#pragma unroll
    for (int x = 0; x < FRT; ++x) {
      const int ins = wid * FRT + x;
      const int row = ins * 8 + (lane >> 3), c = (lane & 7) ^ (row & 7);
      const int voff = (int)(((long)(bm + row) * P.lda + k0 + c * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(stage_a(s) + ins * 1024), 16, voff, 0, 0, 0);
    }
    dma_tile<true>(rb, stage_b(s), P.ldb, bn, k0, wid, lane);
  };

  // deferred stores of the previous tile: packed 16-B values, their rows / columns
  pu32x4 dst[FRT][2];
  int d_bm = 0, d_bn = 0;
  bool d_pending = false;
  // the lane's store of pair (i, jp) of a tile at (bm, bn): row, column
  auto st_row = [&](int bm, int i) { return bm + wm * 16 * FRT + i * 16 + r16; };
  auto st_col = [&](int bn, int jp) { return bn + wn * 64 + 32 * jp + 16 * (q & 1) + 8 * (q >> 1); };
  auto store_one = [&](int idx) {   // idx = i * 2 + jp (compile-time after unrolling)
    const int i = idx >> 1, jp = idx & 1;
    const int m = st_row(d_bm, i), n = st_col(d_bn, jp);
    if (m < P.M && n < P.N) *reinterpret_cast<pu32x4*>(C + (long)m * P.ldc + n) = dst[i][jp];
  };

  int lin = blockIdx.x;
  if (lin >= total) return;
  int bm, bn;
  coords(lin, bm, bn);
  int sc = 0;   // stage of the next k-step (running over tiles)
  dma_stage(0, bm, bn, 0);
  constexpr bool PR = PRIO;
  while (true) {
    f32x4 acc[FRT][4];
#pragma unroll
    for (int i = 0; i < FRT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // stores of the previous tile are spread over k-steps 0 .. nk-2 (none at the last step, whose
    // successor — the next tile's first wait — would have to drain them)
    const int spread = nk > 1 ? nk - 1 : 1;
    int n_prev = 0;   // stores issued in the previous k-step (younger than its DMA)
    for (int kt = 0; kt < nk; ++kt) {
      mmsw::wait_vm_n(n_prev);
      __builtin_amdgcn_s_barrier();
      const int cur = (sc + kt) & 1;
      if (kt + 1 < nk) dma_stage(cur ^ 1, bm, bn, (kt + 1) * BK);
      n_prev = 0;
      if (DEFER && d_pending && nk > 1) {
        // the stores must stay behind the DMA: the next step's counted wait leaves them in flight
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
        const int lo = (kt * NST + spread - 1) / spread, hi = ((kt + 1) * NST + spread - 1) / spread;
#pragma unroll
        for (int idx = 0; idx < NST; ++idx)
          if (idx >= lo && idx < hi) store_one(idx);
        n_prev = (hi < NST ? hi : NST) - lo;
        if (n_prev < 0) n_prev = 0;
      }
      h16x8 fa2[2][FRT], fb2[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < FRT; ++i) fa2[kk][i] = read_frag<true>(stage_a(cur), wm * 16 * FRT + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb2[kk][j] = read_frag<true>(stage_b(cur), wn * 64 + j * 16, kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FRT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb2[kk][j], fa2[kk][i], acc[i][j], 0, 0, 0);
        if (PR) __builtin_amdgcn_s_setprio(0);
      }
    }
    sc += nk;
    // ---- the next tile's first stage into the idle half of the ring (read at k-step nk-2, and
    // every wave has passed the barrier of k-step nk-1 since)
    const int nlin = lin + gridDim.x;
    const bool has_next = nlin < total;
    int nbm = 0, nbn = 0;
    if (has_next) {
      coords(nlin, nbm, nbn);
      dma_stage(sc & 1, nbm, nbn, 0);
    }
    // ---- stores of the previous tile not yet out (nk == 1)
    if (DEFER && d_pending && nk <= 1) {
#pragma unroll
      for (int idx = 0; idx < NST; ++idx) store_one(idx);
    }
    // ---- this tile's epilogue, from the accumulators
    PtDrop D;
    D.fast = false;
    D.hmix = 0;
    D.pbase = 0;
    if (epi_drops<EPI>() && P.thresh) {
      const uint64_t cf = P.offset + (uint64_t)bm * P.ld_rng + bn;
      const uint64_t cl = P.offset + (uint64_t)(bm + BMT - 1) * P.ld_rng + bn + BN - 1;
      D.fast = drop_ok && mms_same_hi(cf, cl);
      D.hmix = mms_hi_mix(P.seed, cf);
      D.pbase = (uint32_t)(cf >> 1);
    }
    float bv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n0 = bn + wn * 64 + 16 * j + 4 * q;
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[j][e] = 0.f;
      if (P.bias && EPI != MMS_EPI_RELU_DROP_BWD && n0 < P.N) {
        const h16x4 b4 = *reinterpret_cast<const h16x4*>(P.bias + n0);
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[j][e] = (float)b4[e];
      }
    }
#pragma unroll
    for (int i = 0; i < FRT; ++i) {
      const int m = bm + wm * 16 * FRT + i * 16 + r16;
      h16x4 ax[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n0 = bn + wn * 64 + 16 * j + 4 * q;
        ax[j] = h16x4{(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
        if (pt_aux<EPI>() && m < P.M && n0 < P.N) ax[j] = *reinterpret_cast<const h16x4*>(P.aux + (long)m * P.ldaux + n0);
      }
      pu32x2 o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n0 = bn + wn * 64 + 16 * j + 4 * q;
        const uint32_t pair0 = D.pbase + (uint32_t)(((m - bm) * (long)P.ld_rng + (n0 - bn)) >> 1);
        o[j] = pt_frag<EPI>(P, acc[i][j], bv[j], ax[j], D, pair0, m, n0, dscale);
      }
      // pair fragments (0, 1) and (2, 3): lane row q ends up with 8 consecutive columns
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const auto s0 = __builtin_amdgcn_permlane16_swap(o[2 * jp][0], o[2 * jp + 1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(o[2 * jp][1], o[2 * jp + 1][1], false, false);
        dst[i][jp] = pu32x4{s0[0], s1[0], s0[1], s1[1]};
      }
    }
    d_bm = bm;
    d_bn = bn;
    d_pending = true;
    if (!DEFER || !has_next) {
#pragma unroll
      for (int idx = 0; idx < NST; ++idx) store_one(idx);
      d_pending = false;
    }
    if (!has_next) break;
    lin = nlin;
    bm = nbm;
    bn = nbn;
  }
  stamp_end(P.stamps, t_start);
}

}  // namespace
}  // namespace mmsp
