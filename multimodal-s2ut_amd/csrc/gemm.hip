// MFMA fp16 GEMM for gfx950 with fused epilogues.
//
//   C[m][n] = epilogue( alpha * sum_k A(m,k) * B(n,k) )
//   A(m,k) = A_KC ? A[m*lda + k] : A[k*lda + m]      (K-contiguous or M-contiguous)
//   B(n,k) = B_KC ? B[n*ldb + k] : B[k*ldb + n]      (K-contiguous or N-contiguous)
//
// One kernel covers every GEMM of the training step: forward projections (NT), dgrad (NN) and
// wgrad (TN), batched attention products (two-level batch strides), split-K for the skinny
// wgrad shapes.  Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 tiles of
// v_mfma_f32_16x16x32_f16.  Operands are register-staged into a double-buffered LDS image:
//   * K-contiguous tile  -> [128 rows][64 k], 16-B chunks XOR-swizzled by (row & 7), read with
//     ds_read_b128 (conflict-free per 16-lane group);
//   * MN-contiguous tile -> [64 k][128 rows], 16-B chunks XOR-swizzled by h(k)<<1, read with the
//     gfx950 transpose read ds_read_b64_tr_b16 (two per fragment), conflict-free per half-wave.
// The MFMA is issued with (B,A) swapped so each lane owns 4 consecutive output columns -> 8-B
// vector stores and 4-wide epilogue math.
#include <stdlib.h>

#include <algorithm>
#include <mutex>

#include "gemm_common.h"

namespace {

#include "gemm_skinny.h"

template <bool KC>
MMS_DEV void load_tile(const h16* __restrict__ X, long ld, int rows_total, int kdim,
                       int row0, int k0, int kend, s16x8 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = t + i * NT;
    s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (KC) {
      const int row = id >> 3, c = id & 7;
      const int gr = row0 + row, gk = k0 + c * 8;
      if (gr < rows_total) {
        const h16* src = X + (long)gr * ld + gk;
        if (gk + 8 <= kend) {
          v = *reinterpret_cast<const s16x8*>(src);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (gk + e < kend) v[e] = reinterpret_cast<const short*>(src)[e];
        }
      }
    } else {
      const int kr = id >> 4, c = id & 15;
      const int gk = k0 + kr, gr = row0 + c * 8;
      if (gk < kend) {
        const h16* src = X + (long)gk * ld + gr;
        if (gr + 8 <= rows_total) {
          v = *reinterpret_cast<const s16x8*>(src);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (gr + e < rows_total) v[e] = reinterpret_cast<const short*>(src)[e];
        }
      }
    }
    r[i] = v;
  }
  (void)kdim;
}

template <bool KC>
MMS_DEV void store_tile(char* lds, const s16x8 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = t + i * NT;
    int off;
    if (KC) {
      const int row = id >> 3, c = id & 7;
      off = row * 128 + ((c ^ (row & 7)) << 4);
    } else {
      const int kr = id >> 4, c = id & 15;
      off = kr * 256 + ((c ^ swz_mn(kr)) << 4);
    }
    *reinterpret_cast<s16x8*>(lds + off) = r[i];
  }
}

template <bool A_KC, bool B_KC, int EPI>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  const int zb = z / P.splitk, zs = z % P.splitk;
  const int z1 = zb / P.bdiv, z2 = zb % P.bdiv;
  const h16* A = P.A + z1 * P.sA1 + z2 * P.sA2;
  const h16* B = P.B + z1 * P.sB1 + z2 * P.sB2;
  const int kbeg = zs * P.kchunk;
  const int kend = min(P.K, kbeg + P.kchunk);
  const int bm = tm * BM, bn = tn * BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // stage s: A image at smem + 2s*TILE_BYTES, B image at smem + (2s+1)*TILE_BYTES
#define SA(s) (smem + (2 * (s)) * TILE_BYTES)
#define SB(s) (smem + (2 * (s) + 1) * TILE_BYTES)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  s16x8 ra[4], rb[4];
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    load_tile<A_KC>(A, P.lda, P.M, P.K, bm, kbeg, kend, ra);
    load_tile<B_KC>(B, P.ldb, P.N, P.K, bn, kbeg, kend, rb);
    store_tile<A_KC>(SA(0), ra);
    store_tile<B_KC>(SB(0), rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      load_tile<A_KC>(A, P.lda, P.M, P.K, bm, k0, kend, ra);
      load_tile<B_KC>(B, P.ldb, P.N, P.K, bn, k0, kend, rb);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      h16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag<A_KC>(SA(cur), wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag<B_KC>(SB(cur), wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<A_KC>(SA(cur ^ 1), ra);
      store_tile<B_KC>(SB(cur ^ 1), rb);
    }
    __syncthreads();
  }
#undef SA
#undef SB

  char* Cz;
  if (EPI == MMS_EPI_F32)
    Cz = reinterpret_cast<char*>(P.C) + (z1 * P.sC1 + z2 * P.sC2 + zs * P.sCsplit) * 4;
  else
    Cz = reinterpret_cast<char*>(P.C) + (z1 * P.sC1 + z2 * P.sC2) * 2;
  const h16* auxz = P.aux ? P.aux + z1 * P.sX1 + z2 * P.sX2 : nullptr;
  staged_epilogue<EPI>(P, smem, acc, bm, bn, wm, wn, wid, lane, Cz, auxz);
  stamp_end(P.stamps, t_start);
}

// ------------------------------------------------------------------------------------------
// LDS-DMA pipelined variant: operands go global -> LDS with buffer_load ... lds (16 B / lane,
// 1 KiB per wave-instruction, no VGPR staging), STAGES-deep ring, counted vmcnt + raw s_barrier
// so the next tiles' DMA stays in flight across the barrier.  The XOR swizzle moves to the
// per-lane SOURCE address (the DMA writes lane-linear LDS), the fragment reads are unchanged.
// Out-of-range rows/k-rows read as zero through the buffer descriptor's range check, so tails
// need no predication; a K-contiguous operand needs K % 64 == 0 (host routing).
// ------------------------------------------------------------------------------------------



// One 128x128 output tile of the LDS-DMA pipeline (z = batch * splitk + split).  PRI: raise the
// wave priority around the MFMA blocks (critical-path GEMMs; not the side stream's weight gradients)
template <bool A_KC, bool B_KC, int EPI, int STAGES, bool RS, bool PRI>
MMS_DEV void dma_gemm_tile(const GemmP& P, char* smem, int z, int tm, int tn) {
  const int zb = z / P.splitk, zs = z % P.splitk;
  const int z1 = zb / P.bdiv, z2 = zb % P.bdiv;
  const int kbeg = zs * P.kchunk;
  const int kend = min(P.K, kbeg + P.kchunk);
  const int bm = tm * BM, bn = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  // buffer descriptors (block-uniform): K-contig base = operand, MN-contig base = row kbeg
  const h16* Ab = P.A + z1 * P.sA1 + z2 * P.sA2 + (A_KC ? 0 : (long)kbeg * P.lda);
  const h16* Bb = P.B + z1 * P.sB1 + z2 * P.sB2 + (B_KC ? 0 : (long)kbeg * P.ldb);
  // exact extents; MN-contiguous rows rounded up to whole 16-B chunks (a chunk straddling the
  // range end would be dropped whole by the range check)
  const long a_ext = A_KC ? ((long)(P.M - 1) * P.lda + P.K) * 2
                          : ((long)(kend - kbeg - 1) * P.lda + ((P.M + 7) & ~7)) * 2;
  const long b_ext = B_KC ? ((long)(P.N - 1) * P.ldb + P.K) * 2
                          : ((long)(kend - kbeg - 1) * P.ldb + ((P.N + 7) & ~7)) * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, (int)a_ext, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, (int)b_ext, 0x00020000);
#define SA(s) (smem + (2 * (s)) * TILE_BYTES)
#define SB(s) (smem + (2 * (s) + 1) * TILE_BYTES)
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // RS: the first column of tiles also sums its A rows over k with one extra MFMA per A fragment
  // (B = ones): lane l ends up with sum_k A(bm + wm*64 + 16i + (l & 15), k) in every element of rs[i]
  f32x4 rs[4];
  const bool do_rs = RS && tn == 0 && wn == 0 && (P.rowsum || P.rowsum16);   // (grouped: db may be NULL)
  if (RS) {
#pragma unroll
    for (int i = 0; i < 4; ++i) rs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  h16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (h16)1.f;
  const int nk = (kend - kbeg + BK - 1) / BK;
  // k offset of stage t relative to the descriptor base
  auto k_rel = [&](int t, bool kc) { return kc ? kbeg + t * BK : t * BK; };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) {
    if (s < nk) {
      dma_tile<A_KC>(ra, SA(s), P.lda, bm, k_rel(s, A_KC), wid, lane);
      dma_tile<B_KC>(rb, SB(s), P.ldb, bn, k_rel(s, B_KC), wid, lane);
    }
  }
  // An MN-contiguous operand is read with ds_read_b64_tr_b16, and the compiler cannot tell those
  // reads from the LDS-DMA writes still in flight: it puts a vmcnt(0) in front of any such read
  // issued after a DMA, which would make every k-step wait for the NEXT stage's DMA to land.  With
  // a transpose-read operand the k-step therefore reads both k-halves' fragments first and issues
  // the next stage's DMA behind them (the DMA then overlaps the MFMAs, as in the K-contiguous form).
#ifndef MMS_GEMM_DMA_AFTER_READS
#define MMS_GEMM_DMA_AFTER_READS 0
#endif
  constexpr bool READ_FIRST = !A_KC || !B_KC || MMS_GEMM_DMA_AFTER_READS;
  // All 16 fragments of the stage are read before its MFMAs (the second k-half's reads no longer
  // wait behind the first half's MFMAs): 0-5 % faster isolated on the step's NT shapes, step flat
  // (profiles/round3_v5_gemm_read_all_ab.txt).
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt must have landed; leave the younger stages (issued earlier) in flight
    const int younger = min(STAGES - 2, nk - 1 - kt);
    if (STAGES >= 3 && younger >= 1) wait_vm<8>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const int nxt = kt + STAGES - 1;
    const int cur = kt % STAGES;
    if (!READ_FIRST && nxt < nk) {
      const int sb = nxt % STAGES;
      dma_tile<A_KC>(ra, SA(sb), P.lda, bm, k_rel(nxt, A_KC), wid, lane);
      dma_tile<B_KC>(rb, SB(sb), P.ldb, bn, k_rel(nxt, B_KC), wid, lane);
    }
    h16x8 fa2[2][4], fb2[2][4];
    {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa2[kk][i] = read_frag<A_KC>(SA(cur), wm * 64 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb2[kk][j] = read_frag<B_KC>(SB(cur), wn * 64 + j * 16, kk, lane);
      }
    }
    if (READ_FIRST && nxt < nk) {
      const int sb = nxt % STAGES;
      dma_tile<A_KC>(ra, SA(sb), P.lda, bm, k_rel(nxt, A_KC), wid, lane);
      dma_tile<B_KC>(rb, SB(sb), P.ldb, bn, k_rel(nxt, B_KC), wid, lane);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      h16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { fa[i] = fa2[kk][i]; fb[i] = fb2[kk][i]; }
      if (PRI) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      if (PRI) __builtin_amdgcn_s_setprio(0);
      if (RS && do_rs) {
#pragma unroll
        for (int i = 0; i < 4; ++i) rs[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, fa[i], rs[i], 0, 0, 0);
      }
    }
  }
#undef SA
#undef SB
  if (RS && do_rs && lane < 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = bm + wm * 64 + i * 16 + lane;
      if (m < P.M) {
        if (P.rowsum16) P.rowsum16[m] = (h16)(rs[i][0] * P.alpha);   // unsplit: the bias gradient itself
        else P.rowsum[(long)zs * P.ld_rowsum + m] = rs[i][0] * P.alpha;   // (do_rs: one of them is set)
      }
    }
  }
  char* Cz;
  if (EPI == MMS_EPI_F32)
    Cz = reinterpret_cast<char*>(P.C) + (z1 * P.sC1 + z2 * P.sC2 + zs * P.sCsplit) * 4;
  else
    Cz = reinterpret_cast<char*>(P.C) + (z1 * P.sC1 + z2 * P.sC2) * 2;
  const h16* auxz = P.aux ? P.aux + z1 * P.sX1 + z2 * P.sX2 : nullptr;
  // the ring is idle once every wave is past its last fragment read (no DMA is in flight: the
  // last k-step waited for vmcnt(0))
  __syncthreads();
#ifdef MMS_GEMM_NOEPI   // ablation build: no epilogue (accumulators kept live; garbage output)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
  (void)Cz; (void)auxz;
#else
  staged_epilogue<EPI>(P, smem, acc, bm, bn, wm, wn, wid, lane, Cz, auxz);
#endif
}

template <bool A_KC, bool B_KC, int EPI, int STAGES, bool RS = false>
__global__ void __launch_bounds__(NT, (STAGES <= 2 ? 2 : 1)) gemm_dma_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[STAGES * 2 * TILE_BYTES];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  dma_gemm_tile<A_KC, B_KC, EPI, STAGES, RS, PRIO && EPI != MMS_EPI_F32>(P, smem, z, tm, tn);
  stamp_end(P.stamps, t_start);
}

// ------------------------------------------------------------------------------------------
// NT tiles of 32 FRT x 128 (FRT = 3: 96 rows, 5: 160, 6: 192): each of the 4 waves owns 16 FRT
// rows (FRT MFMA fragments) x 64 columns; 2-stage LDS-DMA ring of (4 FRT + 16) KiB stages, two
// blocks per CU (192 rows: 80 KiB, exactly half the CU's LDS).  For NT grids just past a round of
// 128x128 tiles (e.g. M = 11-16 k rows x N = 768: 564 tiles of 128 rows for 512 block slots, a
// second round for 52 of them) taller tiles fit fewer rounds at 1.25x / 1.5x the work per tile;
// 96-row tiles fill a short single round better.  Same k order, same MFMA operands per
// accumulator, same staged epilogue per element: bit-identical to gemm_dma_kernel<true, true, EPI, 2>.
// ------------------------------------------------------------------------------------------
template <int EPI, int FRT>
__global__ void __launch_bounds__(NT, 2) gemm_tall_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  constexpr int BMT = 32 * FRT, TILE_T = BMT * 64 * 2;
  // the ring, or the epilogue's 16 KiB staging area per wave if that is larger (96-row tiles)
  constexpr int SMEM = 2 * (TILE_T + TILE_BYTES) > 4 * 64 * 64 * 4 ? 2 * (TILE_T + TILE_BYTES) : 4 * 64 * 64 * 4;
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  (void)z;   // batch 1 (host)
  const int bm = tm * BMT, bn = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const long a_ext = ((long)(P.M - 1) * P.lda + P.K) * 2;
  const long b_ext = ((long)(P.N - 1) * P.ldb + P.K) * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)P.A, (short)0, (int)a_ext, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)P.B, (short)0, (int)b_ext, 0x00020000);
#define SA(s) (smem + (s) * (TILE_T + TILE_BYTES))
#define SB(s) (SA(s) + TILE_T)
  // an A stage of 32 FRT rows: 4 FRT wave-instructions of 8 rows (dma_tile's swizzled layout),
  // FRT per wave; rows past M read as zero through the descriptor
  auto dma_a = [&](char* lds, int k0) {
#ifndef MMS_GEMM_NODMA
#pragma unroll
    for (int x = 0; x < FRT; ++x) {
      const int ins = wid * FRT + x;
      const int row = ins * 8 + (lane >> 3), c = (lane & 7) ^ (row & 7);
      const int voff = (int)(((long)(bm + row) * P.lda + k0 + c * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(lds + ins * 1024), 16, voff, 0, 0, 0);
    }
#endif
  };
  f32x4 acc[FRT][4];
#pragma unroll
  for (int i = 0; i < FRT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = P.K / BK;   // K % 64 == 0 (host)
  if (nk > 0) {
    dma_a(SA(0), 0);
    dma_tile<true>(rb, SB(0), P.ldb, bn, 0, wid, lane);
  }
  constexpr bool PR = PRIO && EPI != MMS_EPI_F32;
  for (int kt = 0; kt < nk; ++kt) {
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      dma_a(SA(cur ^ 1), (kt + 1) * BK);
      dma_tile<true>(rb, SB(cur ^ 1), P.ldb, bn, (kt + 1) * BK, wid, lane);
    }
    h16x8 fa2[2][FRT], fb2[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < FRT; ++i) fa2[kk][i] = read_frag<true>(SA(cur), wm * 16 * FRT + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb2[kk][j] = read_frag<true>(SB(cur), wn * 64 + j * 16, kk, lane);
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
#undef SA
#undef SB
  __syncthreads();   // the ring is idle (the last k-step waited for vmcnt(0))
  // the wave's rows [bm + 16 FRT wm, + 16 FRT): fragments 0-3 (64 rows), then the rest, each
  // through the wave's 16 KiB staging area (staged_epilogue places wave rows at bm + 64 wm)
  constexpr int WR = 16 * FRT, F1 = FRT < 4 ? FRT : 4;
  if constexpr (epi_regs<EPI>() && MMS_GEMM_REG_TALL) {   // all FRT fragments in one pass (fp16 slots: 2 KiB per fragment)
    if (reg_epilogue_ok(P)) {
      reg_epilogue<EPI, FRT, FRT * 2048>(P, smem, acc, bm + (WR - 64) * wm, bn, wm, wn, wid, lane, P.C);
      stamp_end(P.stamps, t_start);
      return;
    }
  }
  staged_epilogue<EPI, F1>(P, smem, reinterpret_cast<const f32x4(&)[F1][4]>(acc[0]), bm + (WR - 64) * wm, bn, wm,
                           wn, wid, lane, P.C, P.aux);
  if constexpr (FRT > 4) {
    __syncthreads();
    staged_epilogue<EPI, FRT - 4>(P, smem, reinterpret_cast<const f32x4(&)[FRT - 4][4]>(acc[4]),
                                  bm + (WR - 64) * wm + 64, bn, wm, wn, wid, lane, P.C, P.aux);
  }
  stamp_end(P.stamps, t_start);
}

// Grouped weight gradients: the dW = dy^T x products of one transformer layer (QKV, out-proj, fc1,
// fc2, and the decoder's cross-attention q / out) as ONE launch over the union of their 128x128
// tiles, unsplit: fp16 dW and (first tile column) fp16 db written straight from the accumulators,
// no fp32 split-K slabs and no reduction pass.  The layer's ~400-500 tiles fill the 512 block slots
// in one round (2 per CU), each tile reducing over all of the layer's token rows.  The linear block
// id is remapped as tile_coords does (each XCD one contiguous range of the grouped tile space),
// then resolved to (problem, tile) by the prefix table.
constexpr int kGroupMax = 8;
struct GemmGroup {
  GemmP p[kGroupMax];
  int first[kGroupMax + 1];   // prefix sums of the problems' tile counts
  int tiles_m[kGroupMax], tiles_n[kGroupMax];
  int n;
  unsigned long long* stamps;
};

// A capped grid (gridDim.x < total, a multiple of 8) walks the tiles persistently: block b takes
// linear tiles b, b + grid, ... — on the side stream the weight gradients then hold at most that
// many of the CUs' block slots, and the critical path's GEMMs keep the rest.
__global__ void __launch_bounds__(NT, 2) gemm_group_wgrad_kernel(GemmGroup G, int total) {
  const unsigned long long t_start = G.stamps ? stamp_now() : 0ull;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES];
  const int q = total / 8, r = total % 8;
  for (int lin = blockIdx.x; lin < total; lin += gridDim.x) {
    if (lin != (int)blockIdx.x) __syncthreads();   // the previous tile's epilogue is done with the ring
    const int x = lin % 8;
    const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lin / 8;
    int g = 0;
    while (g + 1 < G.n && id >= G.first[g + 1]) ++g;
    const GemmP& P = G.p[g];
    const int t = id - G.first[g], tiles_n = G.tiles_n[g];
    const int per_group = P.group_m * tiles_n;
    const int grp = t / per_group, first_m = grp * P.group_m;
    const int gsize = min(G.tiles_m[g] - first_m, P.group_m);
    const int w = t % per_group;
    dma_gemm_tile<false, false, MMS_EPI_F16, 2, true, false>(P, smem, 0, first_m + w % gsize, w / gsize);
  }
  stamp_end(G.stamps, t_start);
}

// ------------------------------------------------------------------------------------------
// 256x256 tile, 8 waves (2 x 4, each 128 rows x 64 cols = 8x4 MFMA tiles), one block per CU.
// 32-deep k-slots in a 4-slot LDS-DMA ring (4 x 32 KiB = 128 KiB): slot ks+3 is issued right
// after the barrier that opens slot ks, so three slots (12 of a wave's DMA instructions) stay in
// flight across every barrier (counted vmcnt, raw s_barrier).  Per slot a wave reads 8 A + 4 B
// fragments and issues 32 MFMAs.  Each 256-row operand image is two 128-row halves in the BK=32
// layouts above.  Epilogue: two 64-row passes through the (idle) ring, 16 KiB per wave.
// ------------------------------------------------------------------------------------------
constexpr int BM2 = 256, BN2 = 256, NT2 = 512, SLOT2 = 2 * 2 * T32_BYTES;  // A 16 KiB + B 16 KiB
constexpr int RING2 = 4;

// one operand's 32-deep slot image: 16 wave-instructions (2 halves x 8); wave w issues w and w+8
template <bool KC>
MMS_DEV void dma_slot2(__amdgpu_buffer_rsrc_t rs, char* img, long ld, int row0, int k0rel, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ins = wid + 8 * i;
    const int half = ins >> 3, hi = ins & 7;
    const int r0 = row0 + half * 128;
    int voff;
    if (KC) {
      const int row = hi * 16 + (lane >> 2), slot = lane & 3;
      const int c = slot ^ swz32(row);
      voff = (int)(((long)(r0 + row) * ld + k0rel + c * 8) * 2);
    } else {
      const int kr = hi * 4 + (lane >> 4), slot = lane & 15;
      const int c = slot ^ swz_mn(kr);
      voff = (int)(((long)(k0rel + kr) * ld + r0 + c * 8) * 2);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + half * T32_BYTES + hi * 1024), 16, voff, 0, 0, 0);
  }
}

// Software-pipelined form of the same tile: each 32-deep slot runs in two MFMA phases (rows
// 0-63, then 64-127 of the wave's 128).  The second half's A fragments are read at the top of the
// slot (behind phase A), and the NEXT slot's first-half A + B fragments are read right after the
// slot's barrier (behind phase B), so no ds_read latency sits in front of an MFMA phase.  A
// RING-slot ring; the barrier of slot s retires slot s+1 (read just after it) and slot s+RING-1
// is issued behind it, leaving RING-3 slots in flight across the barrier.
template <bool A_KC, bool B_KC, int EPI, int RING>
__global__ void __launch_bounds__(NT2, 2) gemm256p_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[RING * SLOT2];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  const int zb = z / P.splitk, zs = z % P.splitk;
  const int z1 = zb / P.bdiv, z2 = zb % P.bdiv;
  const int kbeg = zs * P.kchunk;
  const int kend = min(P.K, kbeg + P.kchunk);
  const int bm = tm * BM2, bn = tn * BN2;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const h16* Ab = P.A + z1 * P.sA1 + z2 * P.sA2 + (A_KC ? 0 : (long)kbeg * P.lda);
  const h16* Bb = P.B + z1 * P.sB1 + z2 * P.sB2 + (B_KC ? 0 : (long)kbeg * P.ldb);
  const long a_ext = A_KC ? ((long)(P.M - 1) * P.lda + P.K) * 2
                          : ((long)(kend - kbeg - 1) * P.lda + ((P.M + 7) & ~7)) * 2;
  const long b_ext = B_KC ? ((long)(P.N - 1) * P.ldb + P.K) * 2
                          : ((long)(kend - kbeg - 1) * P.ldb + ((P.N + 7) & ~7)) * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, (int)a_ext, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, (int)b_ext, 0x00020000);
#define SLA(s) (smem + (s) * SLOT2)
#define SLB(s) (smem + (s) * SLOT2 + 2 * T32_BYTES)
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (kend - kbeg + BK32 - 1) / BK32;
  auto k_rel = [&](int t, bool kc) { return kc ? kbeg + t * BK32 : t * BK32; };
#pragma unroll
  for (int t = 0; t < RING - 1; ++t) {
    if (t < nk) {
      dma_slot2<A_KC>(ra, SLA(t), P.lda, bm, k_rel(t, A_KC), wid, lane);
      dma_slot2<B_KC>(rb, SLB(t), P.ldb, bn, k_rel(t, B_KC), wid, lane);
    }
  }
  const int a_half = wr * T32_BYTES, b_half = (wc >> 1) * T32_BYTES, b_sub = (wc & 1) * 64;
  // counted wait for slot `want` given that slots up to `issued` have been issued (4 DMA each)
  auto wait_slot = [&](int want, int issued) {
    const int younger = min(issued, nk - 1) - want;  // < 0 past the last slot: drain
    if (RING >= 5 && younger >= 3) wait_vm<12>();
    else if (younger >= 2) wait_vm<8>();
    else if (younger == 1) wait_vm<4>();
    else wait_vm<0>();
  };
  // two register sets for the (first-half A, B) fragments, ping-ponged by a 2-way unrolled loop so
  // the next slot's fragments are consumed where they land (no copies, no over-wide lgkm waits)
  h16x8 faA[4], fbA[4], faB[4], fbB[4];
  if (nk > 0) {
    wait_slot(0, RING - 2);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j) fbA[j] = read_frag32<B_KC>(SLB(0) + b_half, b_sub + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) faA[i] = read_frag32<A_KC>(SLA(0) + a_half, i * 16, lane);
  }
  auto slot = [&](int ks, const h16x8 (&fa_lo)[4], const h16x8 (&fb)[4], h16x8 (&fan)[4], h16x8 (&fbn)[4]) {
    const int cur = ks % RING;
    h16x8 fa_hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa_hi[i] = read_frag32<A_KC>(SLA(cur) + a_half, 64 + i * 16, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa_lo[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // slot ks+1 must have landed; slots up to ks+RING-2 are issued at this point.  The wait,
    // barrier and fragment reads run unconditionally (after the last slot they read a stale but
    // valid slot): a conditional read would make hipcc merge lgkm counts across both paths and
    // wait for the next slot's fragments in front of phase B.
    wait_slot(ks + 1, ks + RING - 2);
    __builtin_amdgcn_s_barrier();
    const int nxt = ks + RING - 1;
    if (nxt < nk) {
      const int sn = nxt % RING;
      dma_slot2<A_KC>(ra, SLA(sn), P.lda, bm, k_rel(nxt, A_KC), wid, lane);
      dma_slot2<B_KC>(rb, SLB(sn), P.ldb, bn, k_rel(nxt, B_KC), wid, lane);
    }
    const int c1 = (ks + 1) % RING;
#pragma unroll
    for (int j = 0; j < 4; ++j) fbn[j] = read_frag32<B_KC>(SLB(c1) + b_half, b_sub + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) fan[i] = read_frag32<A_KC>(SLA(c1) + a_half, i * 16, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa_hi[i], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  for (int ks = 0; ks < nk; ks += 2) {
    slot(ks, faA, fbA, faB, fbB);
    if (ks + 1 < nk) slot(ks + 1, faB, fbB, faA, fbA);
  }
#undef SLA
#undef SLB
  char* Cz;
  if (EPI == MMS_EPI_F32)
    Cz = reinterpret_cast<char*>(P.C) + (z1 * P.sC1 + z2 * P.sC2 + zs * P.sCsplit) * 4;
  else
    Cz = reinterpret_cast<char*>(P.C) + (z1 * P.sC1 + z2 * P.sC2) * 2;
  const h16* auxz = P.aux ? P.aux + z1 * P.sX1 + z2 * P.sX2 : nullptr;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  staged_epilogue<EPI>(P, smem, reinterpret_cast<const f32x4(&)[4][4]>(acc[0]), bm + wr * 128, bn + wc * 64,
                       0, 0, wid, lane, Cz, auxz);
  __syncthreads();
  staged_epilogue<EPI>(P, smem, reinterpret_cast<const f32x4(&)[4][4]>(acc[4]), bm + wr * 128 + 64, bn + wc * 64,
                       0, 0, wid, lane, Cz, auxz);
  stamp_end(P.stamps, t_start);
}


// 256x256 tile, software-pipelined, 4-slot ring (the plain form and a 5-slot ring measured slower)
template <bool A_KC, bool B_KC>
int launch_256(int epi, const GemmP& P, int tm, int tn, int nz, hipStream_t s) {
  const int total = tm * tn * nz;
  dim3 grid(total), block(NT2);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm256p_kernel<A_KC, B_KC, E, 4>), grid, block, 0, s, P, tm, tn, total); break;
    MMS_EPI_CASES
#undef CASE
    default: mms::set_error("gemm: bad epilogue %d", epi); return 1;
  }
  return mms::check_launch("gemm256p");
}

// 128x128 tile, LDS-DMA, 2 stages: 64 KiB of LDS, 2 blocks per CU (3 stages at 1 block per CU and
// a BK = 32 four-deep ring both measured slower on the step's shapes, round-2 scripts/gemm_bench.py, git history)
template <bool A_KC, bool B_KC>
int launch_dma(int epi, const GemmP& P, int tm, int tn, int nz, hipStream_t s) {
  const int total = tm * tn * nz;
  dim3 grid(total), block(NT);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_dma_kernel<A_KC, B_KC, E, 2>), grid, block, 0, s, P, tm, tn, total); break;
    MMS_EPI_CASES
#undef CASE
    default: mms::set_error("gemm: bad epilogue %d", epi); return 1;
  }
  return mms::check_launch("gemm_dma2");
}

template <int FRT>
int launch_tall(int epi, const GemmP& P, int tm, int tn, hipStream_t s) {
  const int total = tm * tn;
  dim3 grid(total), block(NT);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_tall_kernel<E, FRT>), grid, block, 0, s, P, tm, tn, total); break;
    MMS_EPI_CASES
#undef CASE
    default: mms::set_error("gemm: bad epilogue %d", epi); return 1;
  }
  return mms::check_launch("gemm_tall");
}

template <bool A_KC, bool B_KC>
int launch_epi(int epi, const GemmP& P, int tm, int tn, int nz, hipStream_t s) {
  const int total = tm * tn * nz;
  dim3 grid(total), block(NT);
  const size_t lds = 0;
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, E>), grid, block, lds, s, P, tm, tn, total); break;
    MMS_EPI_CASES
#undef CASE
    default: mms::set_error("gemm: bad epilogue %d", epi); return 1;
  }
  return mms::check_launch("gemm");
}

// Split-K fixup: sum the alpha-scaled fp32 partials of the splits (split order, so the result does
// not depend on scheduling) and run the unsplit GEMM's epilogue on them -- same bias / residual /
// gate operands and the same dropout counters (m * ld_rng + n), so masks are identical.  One thread
// per 8 columns of a row: 32-B slab reads, 16-B operand loads / stores.
template <int EPI>
__global__ void __launch_bounds__(256) splitk_fixup_kernel(GemmP P, const float* __restrict__ ws, int nsplit) {
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  const int ncg = (P.N + 7) >> 3;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)P.M * ncg) return;   // never thread 0: the grid is ceil(rows * ncg / 256)
  const int m = (int)(i / ncg), n = (int)(i % ncg) * 8;
  const long slab = (long)P.M * P.N;
  const float* src = ws + (long)m * P.N + n;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n + 7 < P.N) {
    for (int s = 0; s < nsplit; ++s) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src + s * slab);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + s * slab + 4);
      v[0] += lo[0]; v[1] += lo[1]; v[2] += lo[2]; v[3] += lo[3];
      v[4] += hi[0]; v[5] += hi[1]; v[6] += hi[2]; v[7] += hi[3];
    }
  } else {
    for (int s = 0; s < nsplit; ++s)
      for (int e = 0; e < 8; ++e)
        if (n + e < P.N) v[e] += src[s * slab + e];
  }
  epilogue_store8<EPI>(P, P.C, P.aux, m, n, v);
  if (P.stamps) {   // no barrier here (threads of the last block may have returned): thread 0's own end
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u64x2*>(P.stamps + 2 * (long)blockIdx.x) = u64x2{t_start, stamp_now()};
    }
  }
}

int launch_fixup(int epi, const GemmP& P, const float* ws, int nsplit, hipStream_t s) {
  const long n = (long)P.M * ((P.N + 7) / 8);
  dim3 grid((unsigned)((n + 255) / 256)), block(256);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((splitk_fixup_kernel<E>), grid, block, 0, s, P, ws, nsplit); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID)
    CASE(MMS_EPI_GATE) CASE(MMS_EPI_RELU_DROP_BWD) CASE(MMS_EPI_F16_ACC) CASE(MMS_EPI_GELU_DROP) CASE(MMS_EPI_GELU_DROP_BWD)
#undef CASE
    default: mms::set_error("gemm: bad epilogue %d for the split-K fixup", epi); return 1;
  }
  return mms::check_launch("splitk_fixup");
}

template <int TM, int TN, int NLOC>
int launch_skinny_t(int epi, const GemmP& P, int nsplit, float* part, int* ticket, int scatter, int* xcc_out,
                    hipStream_t s) {
  const int tm = (P.M + 16 * TM - 1) / (16 * TM), tn = (P.N + 16 * TN - 1) / (16 * TN);
  dim3 grid(8 * ((tm * tn + 7) / 8) * nsplit), block(NT);   // gemm_skinny.h: 8 XCD ranges x splits
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_skinny_kernel<E, TM, TN, NLOC>), grid, block, 0, s, P, tm, tn, nsplit, part, ticket, scatter, xcc_out); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID)
    CASE(MMS_EPI_GATE) CASE(MMS_EPI_RELU_DROP_BWD) CASE(MMS_EPI_F16_ACC) CASE(MMS_EPI_GELU_DROP) CASE(MMS_EPI_GELU_DROP_BWD)
#undef CASE
    default: mms::set_error("gemm: bad epilogue %d for the short-M kernel", epi); return 1;
  }
  return mms::check_launch("gemm_skinny");
}

// (tile code, chunks per wave): 44 = 64x64 tiles (NLOC <= 2: 64 accumulator + 2 x 64 operand VGPRs
// keep two blocks per CU), 24 = 32x64 and 22 = 32x32 (NLOC <= 3)
struct SkinnyPlan { int code = 0, nloc = 0, nsplit = 1; };
// test hook (mms2ut_gemm_set_epilogue): 1 = every epilogue through the fp32 staging (GemmP.vec16 = 3)
int g_epi_staged = 0;
// test hooks (mms2ut_gemm_skinny_debug): deal a tile's splits over different XCDs; record each
// block's hardware XCD id
int g_skinny_scatter = 0;
int* g_skinny_xcc = nullptr;
int launch_skinny(const SkinnyPlan& pl, int epi, const GemmP& P, float* part, int* ticket, hipStream_t s) {
  const int sc = pl.nsplit > 1 ? g_skinny_scatter : 0;
  int* xo = g_skinny_xcc;
  switch (pl.code * 10 + pl.nloc) {
    case 441: return launch_skinny_t<4, 4, 1>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    case 442: return launch_skinny_t<4, 4, 2>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    case 241: return launch_skinny_t<2, 4, 1>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    case 242: return launch_skinny_t<2, 4, 2>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    case 243: return launch_skinny_t<2, 4, 3>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    case 221: return launch_skinny_t<2, 2, 1>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    case 222: return launch_skinny_t<2, 2, 2>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    case 223: return launch_skinny_t<2, 2, 3>(epi, P, pl.nsplit, part, ticket, sc, xo, s);
    default: mms::set_error("gemm: bad short-M plan %d/%d", pl.code, pl.nloc); return 1;
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------
// live GEMM timing (bench roofline): HIP events around every GEMM launch, on its stream
// ------------------------------------------------------------------------------------------
namespace {
struct GemmProfile {
  bool on = false;
  int cap = 0, n = 0;
  hipEvent_t* ev = nullptr;
  // per launch (kept after end() for mms2ut_profile_launches): kernel ms, launched FLOPs, class
  float* l_ms = nullptr;
  double* l_flops = nullptr;
  int* l_cls = nullptr;
  int* l_mnk = nullptr;   // M, N, K, batch*splitk per launch
  double flops = 0.0;
  double bytes = 0.0;  // algorithmic HBM bytes: A, B (and aux / accumulated C) read once, C written once
  // stamp mode (mms2ut_profile_stamps): block stamps instead of events, [2*cursor...) next free slot
  unsigned long long* stamps = nullptr;
  long stamp_cap = 0, cursor = 0;
  long* l_blk = nullptr;  // per launch: first block slot, one past the last (both kernels of a split-K fixup)
} g_prof;

// stamp slots for the next kernel launch of `blocks` workgroups (null when not in stamp mode or full)
unsigned long long* stamp_take(long blocks) {
  if (!g_prof.on || !g_prof.stamps) return nullptr;
  if (g_prof.cursor + blocks > g_prof.stamp_cap) { g_prof.cursor = g_prof.stamp_cap + 1; return nullptr; }
  unsigned long long* p = g_prof.stamps + 2 * g_prof.cursor;
  g_prof.cursor += blocks;
  return p;
}
}  // namespace

extern "C" int mms2ut_profile_begin(int max_launches) {
  MMS_REQUIRE(!g_prof.on, "profile_begin: already active");
  MMS_REQUIRE(max_launches > 0, "profile_begin: max_launches must be > 0");
  g_prof.ev = (hipEvent_t*)calloc(2 * (size_t)max_launches, sizeof(hipEvent_t));
  MMS_REQUIRE(g_prof.ev != nullptr, "profile_begin: out of host memory");
  free(g_prof.l_ms); free(g_prof.l_flops); free(g_prof.l_cls); free(g_prof.l_mnk);
  g_prof.l_mnk = (int*)calloc(4 * (size_t)max_launches, sizeof(int));
  g_prof.l_ms = (float*)calloc((size_t)max_launches, sizeof(float));
  g_prof.l_flops = (double*)calloc((size_t)max_launches, sizeof(double));
  g_prof.l_cls = (int*)calloc((size_t)max_launches, sizeof(int));
  free(g_prof.l_blk);
  g_prof.l_blk = (long*)calloc(2 * (size_t)max_launches, sizeof(long));
  g_prof.stamps = nullptr;
  g_prof.stamp_cap = g_prof.cursor = 0;
  MMS_REQUIRE(g_prof.l_ms && g_prof.l_flops && g_prof.l_cls && g_prof.l_blk, "profile_begin: out of host memory");
  for (int i = 0; i < 2 * max_launches; ++i)
    if (hipEventCreate(&g_prof.ev[i]) != hipSuccess) { mms::set_error("profile_begin: hipEventCreate"); return 1; }
  g_prof.cap = max_launches;
  g_prof.n = 0;
  g_prof.flops = 0.0;
  g_prof.bytes = 0.0;
  g_prof.on = true;
  return 0;
}

extern "C" int mms2ut_profile_end(float* total_ms, int* launches, double* flops) {
  MMS_REQUIRE(g_prof.on, "profile_end: not active");
  g_prof.on = false;
  float tot = 0.f;
  for (int i = 0; i < g_prof.n && !g_prof.stamps; ++i) {
    float ms = 0.f;
    if (hipEventSynchronize(g_prof.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]) != hipSuccess) {
      mms::set_error("profile_end: event timing failed");
      return 1;
    }
    tot += ms;
    g_prof.l_ms[i] = ms;
  }
  for (int i = 0; i < 2 * g_prof.cap; ++i) hipEventDestroy(g_prof.ev[i]);
  free(g_prof.ev);
  g_prof.ev = nullptr;
  if (total_ms) *total_ms = tot;
  if (launches) *launches = g_prof.n;
  if (flops) *flops = g_prof.flops;
  return 0;
}

static int gemm_dispatch(const mms2ut_gemm_args* a, hipStream_t stream);

// tile-rows per L2 group of the tile order (tile_coords); MMS2UT_GEMM_GROUP_M overrides it for
// A/B runs (0: one band of ceil(tiles_m / 8) tile-rows per XCD)
constexpr int kGroupM = 8;
static int group_m_for(int tiles_m) {
  static int env = -2;
  if (env == -2) {
    const char* e = getenv("MMS2UT_GEMM_GROUP_M");
    env = e ? atoi(e) : -1;
  }
  if (env < 0) return kGroupM;
  if (env == 0) return std::max(1, (tiles_m + 7) / 8);
  return env;
}

static int skinny_pick(const mms2ut_gemm_args* a);
static bool short_m_unsplit(const mms2ut_gemm_args* a);

extern "C" int mms2ut_gemm_f16(const mms2ut_gemm_args* a, hipStream_t stream) {
  if (!g_prof.on || g_prof.n >= g_prof.cap) return gemm_dispatch(a, stream);
  const int i = g_prof.n++;
  int rc;
  if (g_prof.stamps) {
    g_prof.l_blk[2 * i] = g_prof.cursor;
    rc = gemm_dispatch(a, stream);
    g_prof.l_blk[2 * i + 1] = g_prof.cursor;   // > stamp_cap: overflowed, not recorded
  } else {
    hipEventRecord(g_prof.ev[2 * i], stream);
    rc = gemm_dispatch(a, stream);
    hipEventRecord(g_prof.ev[2 * i + 1], stream);
  }
  if (a) {
    const double nb = a->batch > 0 ? a->batch : 1;
    const bool skinny = skinny_pick(a) != 0;
    const int nsplit = skinny || short_m_unsplit(a) ? 1 : (a->splitk > 0 ? a->splitk : 1);
    g_prof.flops += 2.0 * a->M * a->N * a->K * nb;
    g_prof.l_flops[i] = 2.0 * a->M * a->N * a->K * nb;
    g_prof.l_mnk[4 * i] = a->M; g_prof.l_mnk[4 * i + 1] = a->N; g_prof.l_mnk[4 * i + 2] = a->K;
    g_prof.l_mnk[4 * i + 3] = (a->batch > 0 ? a->batch : 1) * nsplit;
    g_prof.l_cls[i] = (a->a_kcontig ? 1 : 0) | (a->b_kcontig ? 2 : 0) | (a->epi << 2) | (nb > 1 ? 256 : 0) |
                      ((nsplit > 1 ? 1 : 0) << 9) | (skinny ? 2048 : 0);
    const double c_bytes = (double)a->M * a->N * (a->epi == MMS_EPI_F32 ? 4.0 * (a->splitk > 0 ? a->splitk : 1) : 2.0);
    double extra = 0.0;
    if (a->epi == MMS_EPI_DROP_RESID || a->epi == MMS_EPI_RELU_DROP_BWD || a->epi == MMS_EPI_F16_ACC) extra = 2.0 * a->M * a->N;
    if (a->epi == MMS_EPI_GATE) extra = 6.0 * a->M * a->N;  // o, t read; g written
    g_prof.bytes += nb * (2.0 * ((double)a->M * a->K + (double)a->N * a->K) + c_bytes + extra);
  }
  return rc;
}

static int wgrad_group_dispatch(const mms2ut_wgrad* w, int n, int64_t rows, int max_blocks, hipStream_t stream) {
  MMS_REQUIRE(w && n >= 1 && n <= kGroupMax, "wgrad_group: need 1..%d problems", kGroupMax);
  MMS_REQUIRE(rows >= 0, "wgrad_group: rows < 0");
  GemmGroup G{};
  G.n = n;
  int total = 0;
  for (int i = 0; i < n; ++i) {
    const mms2ut_wgrad& q = w[i];
    MMS_REQUIRE((rows == 0 || (q.dy && q.x)) && q.dW && q.N > 0 && q.K > 0,
                "wgrad_group: problem %d: null operand or empty shape", i);
    MMS_REQUIRE(q.N % 8 == 0 && q.K % 8 == 0 && q.lddy % 8 == 0 && q.ldx % 8 == 0 && q.lddy >= q.N && q.ldx >= q.K,
                "wgrad_group: problem %d: N, K, lddy, ldx must be multiples of 8 (N=%d K=%d)", i, q.N, q.K);
    MMS_REQUIRE(((uintptr_t)q.dy & 15) == 0 && ((uintptr_t)q.x & 15) == 0 && ((uintptr_t)q.dW & 15) == 0 &&
                    (!q.db || ((uintptr_t)q.db & 1) == 0),
                "wgrad_group: problem %d: operands must be 16-B aligned", i);
    MMS_REQUIRE(rows * q.lddy * 2 < (1L << 31) && rows * q.ldx * 2 < (1L << 31),
                "wgrad_group: problem %d: operand extent exceeds a buffer descriptor", i);
    GemmP& P = G.p[i];
    P.A = q.dy; P.B = q.x; P.C = q.dW;
    P.M = q.N; P.N = q.K; P.K = (int)rows;
    P.lda = q.lddy; P.ldb = q.ldx; P.ldc = q.K;
    P.bdiv = 1; P.splitk = 1;
    P.kchunk = (int)((rows + BK - 1) / BK * BK);
    if (P.kchunk == 0) P.kchunk = BK;
    P.alpha = 1.f;
    P.vec16 = g_epi_staged ? 3 : 1;
    P.rowsum16 = q.db;
    P.group_m = kGroupM;
    G.tiles_m[i] = (q.N + BM - 1) / BM;
    G.tiles_n[i] = (q.K + BN - 1) / BN;
    G.first[i] = total;
    total += G.tiles_m[i] * G.tiles_n[i];
  }
  G.first[n] = total;
  if (rows == 0) {   // empty batch: zero gradients (the GEMM's k loop would not run)
    for (int i = 0; i < n; ++i) {
      if (hipMemsetAsync(w[i].dW, 0, (size_t)w[i].N * w[i].K * 2, stream) != hipSuccess ||
          (w[i].db && hipMemsetAsync(w[i].db, 0, (size_t)w[i].N * 2, stream) != hipSuccess)) {
        mms::set_error("wgrad_group: hipMemsetAsync failed");
        return 1;
      }
    }
    return 0;
  }
  int grid = total;
  if (max_blocks > 0 && max_blocks < total) grid = std::max(8, max_blocks / 8 * 8);
  G.stamps = stamp_take(grid);
  hipLaunchKernelGGL(gemm_group_wgrad_kernel, dim3(grid), dim3(NT), 0, stream, G, total);
  return mms::check_launch("gemm_group_wgrad");
}

extern "C" int mms2ut_wgrad_group(const mms2ut_wgrad* w, int n, int64_t rows, int max_blocks, hipStream_t stream) {
  if (!g_prof.on || g_prof.n >= g_prof.cap) return wgrad_group_dispatch(w, n, rows, max_blocks, stream);
  const int i = g_prof.n++;
  int rc;
  if (g_prof.stamps) {
    g_prof.l_blk[2 * i] = g_prof.cursor;
    rc = wgrad_group_dispatch(w, n, rows, max_blocks, stream);
    g_prof.l_blk[2 * i + 1] = g_prof.cursor;
  } else {
    hipEventRecord(g_prof.ev[2 * i], stream);
    rc = wgrad_group_dispatch(w, n, rows, max_blocks, stream);
    hipEventRecord(g_prof.ev[2 * i + 1], stream);
  }
  if (w && n > 0) {
    double fl = 0.0, by = 0.0;
    int sumN = 0;
    for (int j = 0; j < n; ++j) {
      fl += 2.0 * w[j].N * w[j].K * (double)rows;
      by += 2.0 * ((double)rows * (w[j].N + w[j].K) + (double)w[j].N * w[j].K + (w[j].db ? w[j].N : 0));
      sumN += w[j].N;
    }
    g_prof.flops += fl;
    g_prof.bytes += by;
    g_prof.l_flops[i] = fl;
    g_prof.l_mnk[4 * i] = sumN; g_prof.l_mnk[4 * i + 1] = w[0].K; g_prof.l_mnk[4 * i + 2] = (int)rows;
    g_prof.l_mnk[4 * i + 3] = n;
    g_prof.l_cls[i] = (MMS_EPI_F16 << 2) | (1 << 10);   // TN operands (bits 0, 1 clear), grouped
  }
  return rc;
}

extern "C" int mms2ut_profile_launches(float* ms, double* flops, int* cls, int n) {
  MMS_REQUIRE(!g_prof.on && g_prof.l_ms != nullptr, "profile_launches: no finished profile window");
  MMS_REQUIRE(n >= 0 && n <= g_prof.n, "profile_launches: n=%d > %d launches", n, g_prof.n);
  for (int i = 0; i < n; ++i) {
    if (ms) ms[i] = g_prof.l_ms[i];
    if (flops) flops[i] = g_prof.l_flops[i];
    if (cls) cls[i] = g_prof.l_cls[i];
  }
  return 0;
}

extern "C" int mms2ut_profile_shapes(int* mnk, int n) {
  MMS_REQUIRE(!g_prof.on && g_prof.l_mnk != nullptr, "profile_shapes: no finished profile window");
  MMS_REQUIRE(n >= 0 && n <= g_prof.n, "profile_shapes: n=%d > %d launches", n, g_prof.n);
  for (int i = 0; i < 4 * n; ++i) mnk[i] = g_prof.l_mnk[i];
  return 0;
}

// Stamp mode for the open profile window: every GEMM launch records per-block {start, end}
// s_memrealtime ticks into `stamps` (device, 2 x u64 per block, `cap_blocks` blocks) instead of
// HIP events around the launch.  The caller owns the buffer.
extern "C" int mms2ut_profile_stamps(unsigned long long* stamps, long cap_blocks) {
  MMS_REQUIRE(g_prof.on && g_prof.n == 0, "profile_stamps: call right after profile_begin");
  MMS_REQUIRE(stamps != nullptr && cap_blocks > 0 && ((uintptr_t)stamps & 15) == 0, "profile_stamps: bad buffer");
  g_prof.stamps = stamps;
  g_prof.stamp_cap = cap_blocks;
  g_prof.cursor = 0;
  return 0;
}

extern "C" int mms2ut_profile_blocks(long* first_last, int n) {
  MMS_REQUIRE(!g_prof.on && g_prof.l_blk != nullptr, "profile_blocks: no finished profile window");
  MMS_REQUIRE(n >= 0 && n <= g_prof.n, "profile_blocks: n=%d > %d launches", n, g_prof.n);
  for (int i = 0; i < 2 * n; ++i) first_last[i] = g_prof.l_blk[i];
  return 0;
}

extern "C" int mms2ut_wallclock_khz(int* khz) {
  MMS_REQUIRE(khz != nullptr, "wallclock_khz: null");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) {
    mms::set_error("wallclock_khz: hipDeviceGetAttribute failed");
    return 1;
  }
  return 0;
}

extern "C" int mms2ut_profile_bytes(double* bytes) {
  MMS_REQUIRE(bytes != nullptr, "profile_bytes: null");
  *bytes = g_prof.bytes;
  return 0;
}

// Tall NT tiles (gemm_tall_kernel) by a round-count cost: a round of 160-row tiles costs 1.12
// rounds of 128-row ones, a round of 192-row tiles 1.24 (isolated, one-round grids: the taller
// tile reads less B per FLOP; profiles/round4_tall_ab.txt); the cheapest height wins, ties to the
// shorter (mms2ut_gemm_set_tall / env MMS2UT_GEMM_TALL: 1 = by that rule (default), 0 = never,
// 2 / 3 = 160 / 192 rows for every qualifying NT shape).
#ifndef MMS_TALL_C160
#define MMS_TALL_C160 112
#endif
#ifndef MMS_TALL_C192
#define MMS_TALL_C192 124
#endif
#ifndef MMS_TALL_C96   // 96-row tiles: a fuller single round for short grids; <= 0: never by the rule
#define MMS_TALL_C96 89
#endif
// CUs of the current device (cached per device): the block slots a round of tiles fills
static int gemm_cu_count() {
  static int cached[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

static int g_tall_mode = -1;
static int tall_mode() {
  if (g_tall_mode < 0) {
    const char* e = getenv("MMS2UT_GEMM_TALL");
    g_tall_mode = e ? atoi(e) : 1;
  }
  return g_tall_mode;
}
// -> the tile height (160 / 192), 0 = 128-row tiles
static int tall_pick(const mms2ut_gemm_args* a, int tm, int tn) {
  const int mode = tall_mode();
  if (mode == 0) return 0;
  if (mode == 2) return 160;
  if (mode == 3) return 192;
  if (mode == 5) return 96;
  // a round = one block per slot: two blocks per CU (every NT kernel here holds <= 80 KiB of LDS
  // and <= 256 VGPRs at 256 threads)
  const long slots = 2L * gemm_cu_count();
  auto rounds = [&](int bm) { return ((long)((a->M + bm - 1) / bm) * tn + slots - 1) / slots; };
  // costs in hundredths of a 128-row round
  const long c128 = 100 * rounds(128), c160 = MMS_TALL_C160 * rounds(160), c192 = MMS_TALL_C192 * rounds(192);
  // 96-row tiles were measured on single-round grids of M = 4-7 k rows (profiles/round4_tall_ab.txt);
  // below ~3 k rows (short batches, decode) the 128-row tile keeps the rule's measured range
  const long c96 = MMS_TALL_C96 > 0 && a->M >= 3072 ? MMS_TALL_C96 * rounds(96) : 1L << 40;
  int best = 0;
  long cb = c128;
  if (c160 < cb) { best = 160; cb = c160; }
  if (c192 < cb) { best = 192; cb = c192; }
  if (c96 < cb) { best = 96; cb = c96; }
  return best;
}
extern "C" int mms2ut_gemm_set_tall(int mode) {
  MMS_REQUIRE(mode >= 0 && mode <= 5 && mode != 4, "gemm_set_tall: mode must be 0..3 or 5 (got %d)", mode);
  g_tall_mode = mode;
  return 0;
}

// Short-M NT GEMMs (gemm_skinny.h): those whose 128x128 grid would cover fewer than 128 tiles
// (the decoder's ~470-row projections and the fusion's short image rows), which otherwise take the
// split-K + fixup route.  The plan minimises a latency model of the kernel: the busiest CU's
// operand bytes at ~60 GB/s per CU (the rate a block's one-shot VGPR loads were measured to
// draw), plus, with a K split, the partial-tile round trip and the last block's reduction reads.
// A split needs the caller's split-K workspace (splitk_ws) and the stream's ticket array.
// MMS2UT_GEMM_SKINNY / mms2ut_gemm_set_skinny: 1 = the measured route table below (default),
// 0 = the split-K + fixup route as the caller asked (A/B), 2 = this kernel for every short-M shape.
static int g_skinny_mode = -1;
static int skinny_mode() {
  if (g_skinny_mode < 0) {
    const char* e = getenv("MMS2UT_GEMM_SKINNY");
    g_skinny_mode = e ? atoi(e) : 1;
  }
  return g_skinny_mode;
}
constexpr int kTicketCap = 2048;   // tiles per launch with a K split (every short-M grid of 32x32 tiles fits)
static bool skinny_eligible(const mms2ut_gemm_args* a) {
  if (!skinny_mode() || !a || !a->a_kcontig || !a->b_kcontig || a->batch != 1 || a->epi == MMS_EPI_F32 ||
      a->rowsum || a->K <= 0 || a->K % 256 || a->M <= 0 || a->N <= 0)
    return false;
  if ((long)((a->M + 127) / 128) * ((a->N + 127) / 128) >= 128) return false;
  // measured route table (profiles/round5_short_m_gemm.txt, M = 470 / 900 decoder shapes): the
  // short-M kernel wins for N <= 1024 (K = 768 at any M; K = 2304-3072 at M <= ~600); the 128-row
  // tiles unsplit win for N >= 1536 at K <= 1024; the split-K + fixup route keeps the rest
  return skinny_mode() == 2 || (a->N <= 1024 && (a->M <= 640 || a->K <= 1024));
}
// a short-M fused-epilogue GEMM whose caller asked for the split-K fixup but that runs faster on
// the unsplit 128-row tiles (wide N, short K: enough tiles already)
static bool short_m_unsplit(const mms2ut_gemm_args* a) {
  return skinny_mode() == 1 && a && a->a_kcontig && a->b_kcontig && a->batch == 1 && a->epi != MMS_EPI_F32 &&
         a->splitk > 1 && a->N > 1024 && a->K <= 1024;
}
// The partial-tile workspace a split plan may use: what every caller of the split-K fixup sizes
// (kernels.py _fixup_splits / layers.hip fixup_splits: s * M * N floats), so the plan — and the bits —
// do not depend on which caller (or how large a workspace) issued the GEMM.
static double skinny_ws_budget(const mms2ut_gemm_args* a) {
  if (a->N % 4 || a->K < 512) return 0.0;
  const long tiles = (long)((a->M + 127) / 128) * ((a->N + 127) / 128);
  const long s = std::max(1L, std::min(std::min(512L / tiles, (long)a->K / 256), 16L));
  if (s < 2 || !a->splitk_ws || a->splitk_ws_floats < s * a->M * (long)a->N) return 0.0;
  return (double)s * a->M * a->N;
}
static SkinnyPlan skinny_plan(const mms2ut_gemm_args* a, bool can_split) {
  SkinnyPlan best;
  if (!skinny_eligible(a)) return best;
  const double ws_budget = skinny_ws_budget(a);
  const long cus = gemm_cu_count();
  const int kq = a->K / 256;                  // 256-wide k quarters: one 64-chunk per wave
  double best_t = 1e30;
  const int codes[3] = {44, 24, 22};
  for (int code : codes) {
    const int bm = 16 * (code / 10), bn = 16 * (code % 10);
    const long tiles = (long)((a->M + bm - 1) / bm) * ((a->N + bn - 1) / bn);
    for (int nloc = (code == 44 ? 2 : 3); nloc >= 1; --nloc) {
      if (kq % nloc) continue;
      const int S = kq / nloc;
      if (S > 16 || (S > 1 && (!can_split || tiles > kTicketCap ||
                               (double)tiles * S * bm * bn > ws_budget)))
        continue;
      const long blocks = tiles * S;
      const double per_cu = (double)((blocks + cus - 1) / cus);
      const double bytes = (double)(bm + bn) * 256.0 * nloc * 2.0;
      double t = per_cu * bytes / 60e3;                               // us at 60 GB/s per CU
      if (S > 1) t += 2.5 + (double)S * bm * bn * 4.0 / 60e3;       // partial round trip + reduction reads
      if (t < best_t) { best_t = t; best.code = code; best.nloc = nloc; best.nsplit = S; }
    }
  }
  return best;
}
// Ticket arrays of the split plans: one 8 KiB slice (kTicketCap tiles) per (device, stream) out of
// a per-device pool allocated and zeroed once, on the first split launch of the device; every
// completed launch leaves its slice zero (the reducers re-arm their tickets), a failed launch gets
// its slice re-zeroed in stream order.  Slices are handed out under a mutex (autograd's device
// thread and the main thread both issue GEMMs).  A stream that first needs a slice while the device
// has no pool yet and the stream is capturing cannot get one: that launch fails loudly (the plan —
// and so the bits — never depends on whether tickets exist).
constexpr int kTicketSlices = 512;
static int* skinny_tickets(hipStream_t stream) {
  static std::mutex mu;
  struct Slot { int dev; hipStream_t s; };
  static int* pool[16] = {nullptr};
  static Slot slots[16][kTicketSlices];
  static int used[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) {
    mms::set_error("gemm: short-M split tickets: no current device");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < used[dev]; ++i)
    if (slots[dev][i].s == stream) return pool[dev] + (long)i * kTicketCap;
  if (!pool[dev]) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone) {
      mms::set_error("gemm: short-M split tickets are allocated on the device's first split launch, which must "
                     "not be inside a stream capture (run the step eagerly once first)");
      return nullptr;
    }
    int* p = nullptr;
    const size_t bytes = (size_t)kTicketSlices * kTicketCap * sizeof(int);
    if (hipMalloc(&p, bytes) != hipSuccess || hipMemset(p, 0, bytes) != hipSuccess) {
      if (p) (void)hipFree(p);
      mms::set_error("gemm: short-M split tickets: allocation failed");
      return nullptr;
    }
    pool[dev] = p;
  }
  if (used[dev] == kTicketSlices) {
    mms::set_error("gemm: short-M split tickets: more than %d streams on device %d", kTicketSlices, dev);
    return nullptr;
  }
  slots[dev][used[dev]] = Slot{dev, stream};
  return pool[dev] + (long)(used[dev]++) * kTicketCap;
}
static int skinny_pick(const mms2ut_gemm_args* a) { return skinny_plan(a, a && a->splitk_ws).code; }
extern "C" int mms2ut_gemm_skinny_debug(int scatter, int* xcc_out) {
  g_skinny_scatter = scatter ? 1 : 0;
  g_skinny_xcc = xcc_out;
  return 0;
}
extern "C" int mms2ut_gemm_set_epilogue(int staged) {
  g_epi_staged = staged ? 1 : 0;
  return 0;
}
extern "C" int mms2ut_gemm_set_skinny(int mode) {
  MMS_REQUIRE(mode >= 0 && mode <= 2, "gemm_set_skinny: mode must be 0, 1 or 2 (got %d)", mode);
  g_skinny_mode = mode;
  return 0;
}

// 256x256-tile kernel or the 128x128 one
static bool use_256(const mms2ut_gemm_args* a, int nz) {
  static int force = -2;   // MMS2UT_GEMM_256=1 / 0: every / no eligible shape on the 256 tile (A/B)
  if (force == -2) {
    const char* e = getenv("MMS2UT_GEMM_256");
    force = e ? atoi(e) : -1;
  }
  if (force >= 0) return force == 1 && nz == 1;
  // measured (round-2 A/B, scripts/gemm_ab.py in git history): the 256 tile wins only with a long K and enough tiles to keep
  // one block per CU busy (subsampler conv2, large squares); the step's K = 768 projections and
  // every N = 768 shape run faster on 128x128 tiles at two blocks per CU
  return nz == 1 && a->K >= 2048 && a->N >= 1536 && a->M >= 4096;
}

static int gemm_dispatch(const mms2ut_gemm_args* a, hipStream_t stream) {
  MMS_REQUIRE(a != nullptr, "gemm: null args");
  MMS_REQUIRE(a->M >= 0 && a->N >= 0 && a->K >= 0, "gemm: negative dims");
  if (a->M == 0 || a->N == 0 || a->batch == 0) return 0;
  MMS_REQUIRE(a->lda % 8 == 0 && a->ldb % 8 == 0, "gemm: lda/ldb must be multiples of 8 (lda=%ld ldb=%ld)", a->lda, a->ldb);
  MMS_REQUIRE(((uintptr_t)a->A & 15) == 0 && ((uintptr_t)a->B & 15) == 0, "gemm: A/B must be 16-byte aligned");
  MMS_REQUIRE(a->epi == MMS_EPI_F32 ? (a->ldc % 4 == 0) : (a->ldc % 4 == 0), "gemm: ldc must be a multiple of 4");
  const bool a_kc = a->a_kcontig != 0, b_kc = a->b_kcontig != 0;
  // strides must keep 16-B alignment for every batch
  MMS_REQUIRE(a->sA1 % 8 == 0 && a->sA2 % 8 == 0 && a->sB1 % 8 == 0 && a->sB2 % 8 == 0, "gemm: batch strides must be multiples of 8");
  GemmP P{};
  P.A = a->A; P.B = a->B; P.C = a->C;
  P.M = a->M; P.N = a->N; P.K = a->K;
  P.lda = a->lda; P.ldb = a->ldb; P.ldc = a->ldc;
  P.bdiv = a->bdiv > 0 ? a->bdiv : 1;
  P.sA1 = a->sA1; P.sA2 = a->sA2; P.sB1 = a->sB1; P.sB2 = a->sB2; P.sC1 = a->sC1; P.sC2 = a->sC2;
  int splitk = a->splitk > 0 ? a->splitk : 1;
  if (splitk > 1 && a->epi != MMS_EPI_F32 && skinny_pick(a)) {
    mms2ut_gemm_args b = *a;   // the caller's split-K request is the fallback route; its workspace
    b.splitk = 1;              // holds the short-M kernel's partial tiles
    return gemm_dispatch(&b, stream);
  }
  if (short_m_unsplit(a)) {
    mms2ut_gemm_args b = *a;
    b.splitk = 1; b.splitk_ws = nullptr; b.splitk_ws_floats = 0;
    return gemm_dispatch(&b, stream);
  }
  if (splitk > 1 && a->epi != MMS_EPI_F32) {
    // split-K + fixup: the splits as an fp32-slab GEMM into the workspace, then the epilogue pass
    MMS_REQUIRE(a->batch == 1 && !a->rowsum && a->N % 4 == 0, "gemm: split-K fixup needs batch 1, N %% 4 == 0");
    MMS_REQUIRE(a->splitk_ws && a->splitk_ws_floats >= (int64_t)splitk * a->M * a->N,
                "gemm: split-K fixup workspace too small (%ld floats for %d x %d x %d)",
                (long)a->splitk_ws_floats, splitk, a->M, a->N);
    MMS_REQUIRE(((uintptr_t)a->splitk_ws & 15) == 0, "gemm: split-K workspace must be 16-B aligned");
    mms2ut_gemm_args b = *a;
    b.C = a->splitk_ws; b.ldc = a->N; b.sC1 = b.sC2 = 0; b.sCsplit = (int64_t)a->M * a->N;
    b.epi = MMS_EPI_F32; b.bias = nullptr; b.aux = nullptr; b.out2 = nullptr; b.dropout_p = 0.f;
    b.splitk_ws = nullptr;
    const int rc = gemm_dispatch(&b, stream);
    if (rc) return rc;
    GemmP F{};
    F.C = a->C; F.M = a->M; F.N = a->N; F.K = a->K; F.ldc = a->ldc;
    F.alpha = 1.f; F.bias = a->bias;
    F.aux = a->aux; F.ldaux = a->ldaux; F.out2 = a->out2; F.ldo2 = a->ldo2;
    F.p = a->dropout_p; F.thresh = mms_drop_thresh(a->dropout_p); F.seed = a->seed; F.offset = a->offset;
    F.ld_rng = a->ld_rng > 0 ? a->ld_rng : a->N;
    MMS_REQUIRE(!(a->epi == MMS_EPI_DROP_RESID || a->epi == MMS_EPI_GATE || a->epi == MMS_EPI_GELU_DROP_BWD) || a->aux,
                "gemm: epilogue needs aux");
    MMS_REQUIRE(a->epi != MMS_EPI_RELU_DROP_BWD || a->aux, "gemm: RELU_DROP_BWD needs aux");
    MMS_REQUIRE(!(a->epi == MMS_EPI_GATE || a->epi == MMS_EPI_GELU_DROP) || a->out2, "gemm: epilogue needs out2");
    MMS_REQUIRE(a->ldc % 4 == 0 && (!a->aux || (a->ldaux % 4 == 0 && ((uintptr_t)a->aux & 7) == 0)) &&
                (!a->bias || ((uintptr_t)a->bias & 7) == 0), "gemm: fixup operand alignment");
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    bool v = al16(a->C) && a->ldc % 8 == 0;
    if (a->aux) v = v && al16(a->aux) && a->ldaux % 8 == 0 && (a->epi != MMS_EPI_GATE || a->N % 8 == 0);
    if (a->out2) v = v && al16(a->out2) && a->ldo2 % 8 == 0;
    if (a->bias) v = v && al16(a->bias);
    F.vec16 = v ? (g_epi_staged ? 3 : 1) : 0;
    F.stamps = stamp_take(((long)a->M * ((a->N + 7) / 8) + 255) / 256);
    return launch_fixup(a->epi, F, a->splitk_ws, splitk, stream);
  }
  MMS_REQUIRE(splitk == 1 || a->epi == MMS_EPI_F32, "gemm: split-K needs the fp32 slab epilogue");
  int kchunk = (a->K + splitk - 1) / splitk;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  if (kchunk == 0) kchunk = BK;
  P.splitk = splitk; P.kchunk = kchunk; P.sCsplit = a->sCsplit;
  P.alpha = a->alpha; P.bias = a->bias;
  P.aux = a->aux; P.ldaux = a->ldaux; P.sX1 = a->sX1; P.sX2 = a->sX2;
  P.out2 = a->out2; P.ldo2 = a->ldo2;
  P.p = a->dropout_p; P.thresh = mms_drop_thresh(a->dropout_p); P.seed = a->seed; P.offset = a->offset;
  P.ld_rng = a->ld_rng > 0 ? a->ld_rng : a->N;
  P.group_m = group_m_for((a->M + BM - 1) / BM);
  MMS_REQUIRE(!(a->epi == MMS_EPI_DROP_RESID || a->epi == MMS_EPI_GATE || a->epi == MMS_EPI_GELU_DROP_BWD) || a->aux,
              "gemm: epilogue needs aux");
  MMS_REQUIRE(a->epi != MMS_EPI_RELU_DROP_BWD || a->aux, "gemm: RELU_DROP_BWD needs aux");
  MMS_REQUIRE(!(a->epi == MMS_EPI_GATE || a->epi == MMS_EPI_GELU_DROP) || a->out2, "gemm: epilogue needs out2");
  {
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    bool v = al16(a->C) && a->ldc % 8 == 0 && a->sC1 % 8 == 0 && a->sC2 % 8 == 0;
    if (a->aux) v = v && al16(a->aux) && a->ldaux % 8 == 0 && a->sX1 % 8 == 0 && a->sX2 % 8 == 0 &&
                    (a->epi != MMS_EPI_GATE || a->N % 8 == 0);
    if (a->out2) v = v && al16(a->out2) && a->ldo2 % 8 == 0;
    if (a->bias) v = v && al16(a->bias);
    P.vec16 = v ? (g_epi_staged ? 3 : 1) : 0;
  }
  if (splitk == 1 && skinny_eligible(a)) {
    const SkinnyPlan pl = skinny_plan(a, a->splitk_ws != nullptr);
    if (pl.code) {
      int* tickets = nullptr;
      if (pl.nsplit > 1 && !(tickets = skinny_tickets(stream))) return 1;
      const int q = pl.code / 10, r = pl.code % 10;
      const long tiles = (long)((a->M + 16 * q - 1) / (16 * q)) * ((a->N + 16 * r - 1) / (16 * r));
      P.stamps = stamp_take(8 * ((tiles + 7) / 8) * pl.nsplit);
      const int rc = launch_skinny(pl, a->epi, P, pl.nsplit > 1 ? a->splitk_ws : nullptr, tickets, stream);
      if (rc && tickets) (void)hipMemsetAsync(tickets, 0, kTicketCap * sizeof(int), stream);   // re-arm after a failure
      return rc;
    }
  }
  const int tm = (a->M + BM - 1) / BM, tn = (a->N + BN - 1) / BN;
  const int nz = a->batch * splitk;
  MMS_REQUIRE((long)tm * tn * nz < (1L << 31), "gemm: too many tiles");
  hipStream_t s = stream;
  // LDS-DMA pipeline when every K-contiguous operand has whole 64-wide k-tiles and the operand
  // extents fit a buffer descriptor; otherwise the register-staged kernel (predicated tails)
  MMS_REQUIRE(!a->aux || (a->ldaux % 4 == 0 && ((uintptr_t)a->aux & 7) == 0), "gemm: aux must be 8-B aligned with ldaux %% 4 == 0");
  MMS_REQUIRE(!a->bias || ((uintptr_t)a->bias & 7) == 0, "gemm: bias must be 8-B aligned");
  const bool k_ok = (!a_kc || a->K % BK == 0) && (!b_kc || a->K % BK == 0);
  const long a_ext = a_kc ? (long)a->M * a->lda : (long)a->K * a->lda;
  const long b_ext = b_kc ? (long)a->N * a->ldb : (long)a->K * a->ldb;
  const bool dma_ok = k_ok && a_ext * 2 < (1L << 31) && b_ext * 2 < (1L << 31);
  if (a->rowsum) {
    MMS_REQUIRE(a->epi == MMS_EPI_F32 && !a_kc && !b_kc && a->batch == 1 && dma_ok,
                "gemm: rowsum needs the fp32 slab epilogue, M/N-contiguous operands, batch 1");
    MMS_REQUIRE(a->ld_rowsum >= a->M, "gemm: ld_rowsum < M");
    P.rowsum = a->rowsum; P.ld_rowsum = a->ld_rowsum;
    P.stamps = stamp_take((long)tm * tn * nz);
    dim3 grid(tm * tn * nz), block(NT);
    hipLaunchKernelGGL((gemm_dma_kernel<false, false, MMS_EPI_F32, 2, true>), grid, block, 0, s, P, tm, tn, tm * tn * nz);
    return mms::check_launch("gemm_dma_rs");
  }
  if (dma_ok && a_kc && b_kc && nz == 1) {
    if (const int bmt = tall_pick(a, tm, tn)) {
      const int tmt = (a->M + bmt - 1) / bmt;
      P.group_m = group_m_for(tmt);
      P.stamps = stamp_take((long)tmt * tn);
      if (bmt == 96) return launch_tall<3>(a->epi, P, tmt, tn, s);
      return bmt == 160 ? launch_tall<5>(a->epi, P, tmt, tn, s) : launch_tall<6>(a->epi, P, tmt, tn, s);
    }
  }
  if (dma_ok) {
    if (use_256(a, nz)) {
      const int tm2 = (a->M + BM2 - 1) / BM2, tn2 = (a->N + BN2 - 1) / BN2;
      P.stamps = stamp_take((long)tm2 * tn2 * nz);
      if (a_kc && b_kc) return launch_256<true, true>(a->epi, P, tm2, tn2, nz, s);
      if (a_kc && !b_kc) return launch_256<true, false>(a->epi, P, tm2, tn2, nz, s);
      if (!a_kc && b_kc) return launch_256<false, true>(a->epi, P, tm2, tn2, nz, s);
      return launch_256<false, false>(a->epi, P, tm2, tn2, nz, s);
    }
    P.stamps = stamp_take((long)tm * tn * nz);
    if (a_kc && b_kc) return launch_dma<true, true>(a->epi, P, tm, tn, nz, s);
    if (a_kc && !b_kc) return launch_dma<true, false>(a->epi, P, tm, tn, nz, s);
    if (!a_kc && b_kc) return launch_dma<false, true>(a->epi, P, tm, tn, nz, s);
    return launch_dma<false, false>(a->epi, P, tm, tn, nz, s);
  }
  P.stamps = stamp_take((long)tm * tn * nz);
  if (a_kc && b_kc) return launch_epi<true, true>(a->epi, P, tm, tn, nz, s);
  if (a_kc && !b_kc) return launch_epi<true, false>(a->epi, P, tm, tn, nz, s);
  if (!a_kc && b_kc) return launch_epi<false, true>(a->epi, P, tm, tn, nz, s);
  return launch_epi<false, false>(a->epi, P, tm, tn, nz, s);
}

namespace mms {
int bind_step_seed_gemm(const uint64_t* d) { return mms_bind_step_seed_tu(d); }
}  // namespace mms
