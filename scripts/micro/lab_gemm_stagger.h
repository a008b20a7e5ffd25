// Persistent tall NT GEMM with a staggered second block per CU (gfx950 lab, round 6).
//
// Why: two blocks share each CU (grid 512 = 256 CUs x 2; the census shows block b and b + 256 on
// one CU) and run the same k-loop in lockstep, so both reach their epilogue together: every CU
// stops issuing MFMAs while the chip writes C in one burst.  Here the blocks of the second half of
// the grid (role 1) wait `stag` s_memrealtime ticks before their first tile, so on every CU one
// block's epilogue falls inside the other's k-loop.  The static walk (tile b, b + grid, ...) gives
// the extra tiles of a partial last round to the low block ids, i.e. to role 0, which started
// earlier.  The k-loop and epilogue are gemm_tall_kernel's, so C is bit-identical to it; the
// stagger changes timing only (a different placement only changes speed).
#pragma once

namespace mmst {
namespace {

// MODE 0: the staged epilogue; 2: no epilogue (accumulators kept live); 3: raw accumulators stored
// straight from the MFMA layout as fp16 (8-B stores, no LDS staging, no epilogue math)
template <int EPI, int FRT, int MODE>
__global__ void __launch_bounds__(NT, 2) gemm_stag_kernel(GemmP P, int tiles_m, int tiles_n, int total, int stag) {
  constexpr int BMT = 32 * FRT, TILE_T = BMT * 64 * 2;
  constexpr int SMEM = 2 * (TILE_T + TILE_BYTES) > 4 * 64 * 64 * 4 ? 2 * (TILE_T + TILE_BYTES) : 4 * 64 * 64 * 4;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  if (stag > 0 && (int)blockIdx.x >= (int)gridDim.x / 2) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)stag) __builtin_amdgcn_s_sleep(4);
  }
  const long a_ext = ((long)(P.M - 1) * P.lda + P.K) * 2;
  const long b_ext = ((long)(P.N - 1) * P.ldb + P.K) * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)P.A, (short)0, (int)a_ext, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)P.B, (short)0, (int)b_ext, 0x00020000);
  const int nk = P.K / BK;
  for (int lin = blockIdx.x; lin < total; lin += gridDim.x) {
    if (lin != (int)blockIdx.x) __syncthreads();
    int z, tm, tn;
    tile_coords(lin, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
    const int bm = tm * BMT, bn = tn * BN;
#define SA(s) (smem + (s) * (TILE_T + TILE_BYTES))
#define SB(s) (SA(s) + TILE_T)
    auto dma_a = [&](char* lds, int k0) {
#pragma unroll
      for (int x = 0; x < FRT; ++x) {
        const int ins = wid * FRT + x;
        const int row = ins * 8 + (lane >> 3), c = (lane & 7) ^ (row & 7);
        const int voff = (int)(((long)(bm + row) * P.lda + k0 + c * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(lds + ins * 1024), 16, voff, 0, 0, 0);
      }
    };
    f32x4 acc[FRT][4];
#pragma unroll
    for (int i = 0; i < FRT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    dma_a(SA(0), 0);
    dma_tile<true>(rb, SB(0), P.ldb, bn, 0, wid, lane);
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
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FRT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb2[kk][j], fa2[kk][i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
#undef SA
#undef SB
    if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < FRT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
      continue;
    }
    if (MODE == 3) {
      h16* C = reinterpret_cast<h16*>(P.C);
#pragma unroll
      for (int i = 0; i < FRT; ++i) {
        const int m = bm + wm * 16 * FRT + 16 * i + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = bn + wn * 64 + 16 * j + 4 * (lane >> 4);
          if (m < P.M && n < P.N)
            *reinterpret_cast<h16x4*>(C + (long)m * P.ldc + n) =
                h16x4{(h16)acc[i][j][0], (h16)acc[i][j][1], (h16)acc[i][j][2], (h16)acc[i][j][3]};
        }
      }
      continue;
    }
    __syncthreads();
    constexpr int WR = 16 * FRT, F1 = FRT < 4 ? FRT : 4;
    staged_epilogue<EPI, F1>(P, smem, reinterpret_cast<const f32x4(&)[F1][4]>(acc[0]), bm + (WR - 64) * wm, bn, wm,
                             wn, wid, lane, P.C, P.aux);
    if constexpr (FRT > 4) {
      __syncthreads();
      staged_epilogue<EPI, FRT - 4>(P, smem, reinterpret_cast<const f32x4(&)[FRT - 4][4]>(acc[4]),
                                    bm + (WR - 64) * wm + 64, bn, wm, wn, wid, lane, P.C, P.aux);
    }
  }
}

template <int FRT, int MODE>
int launch_stag_t(int epi, const GemmP& P, hipStream_t s, int stag) {
  constexpr int BMT = 32 * FRT;
  const int tm = (P.M + BMT - 1) / BMT, tn = (P.N + 127) / 128, total = tm * tn;
  const int grid = total < 512 ? total : 512;
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_stag_kernel<E, FRT, MODE>), dim3(grid), dim3(NT), 0, s, P, tm, tn, total, stag); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_RELU_DROP_BWD)
#undef CASE
    default: return 1;
  }
  return hipGetLastError() != hipSuccess;
}

// bm: tile height (96 / 128 / 160 / 192); var = frac100 + 1000 * MODE, frac100: the stagger as
// hundredths of an estimated paired tile time (25 us for a 192-row tile at K = 768, scaled by K and
// height)
template <int MODE>
int launch_stag_m(int epi, int bm, int frac100, const GemmP& P, hipStream_t s) {
  const double tile_us = 25.0 * (P.K / 768.0) * (bm / 192.0);
  const int stag = (int)(tile_us * frac100 / 100.0 * 100.0);   // s_memrealtime: 100 MHz
  if (bm == 192) return launch_stag_t<6, MODE>(epi, P, s, stag);
  if (bm == 160) return launch_stag_t<5, MODE>(epi, P, s, stag);
  if (bm == 128) return launch_stag_t<4, MODE>(epi, P, s, stag);
  return 1;
}
int launch_stag(int epi, int bm, int var, const GemmP& P, hipStream_t s) {
  const int mode = var / 1000, frac = var % 1000;
  if (mode == 2) return launch_stag_m<2>(epi, bm, frac, P, s);
  if (mode == 3) return launch_stag_m<3>(epi, bm, frac, P, s);
  return launch_stag_m<0>(epi, bm, frac, P, s);
}

}  // namespace
}  // namespace mmst

// ---------------------------------------------------------------------------------------------
// MODE 4 (round 6): persistent tall kernel that prefetches the NEXT tile's first k-stage during the
// current tile's epilogue.  The epilogue stages 32 rows per wave per pass (8 KiB slots, the ring's
// first 32 KiB), so ring stage 1 (bytes 40-80 KiB at 192 rows) is free: the next tile's k = 0 stage
// is issued into it right after the k-loop, and every tile's k-loop starts at stage 1.  The first
// k-step then waits for the prefetch only (vmcnt counted past the epilogue's stores) on full tiles.
// Same k order and epilogue arithmetic as gemm_tall_kernel: bit-identical.
// ---------------------------------------------------------------------------------------------
namespace mmst {
namespace {
template <int EPI, int FRT>
__global__ void __launch_bounds__(NT, 2) gemm_pf_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  constexpr int BMT = 32 * FRT, TILE_T = BMT * 64 * 2;
  constexpr int SMEM = 2 * (TILE_T + TILE_BYTES);
  static_assert(4 * 32 * 64 * 4 <= TILE_T + TILE_BYTES, "staging must fit ring stage 0");
  static_assert(FRT % 2 == 0, "2-fragment epilogue passes");
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const long a_ext = ((long)(P.M - 1) * P.lda + P.K) * 2;
  const long b_ext = ((long)(P.N - 1) * P.ldb + P.K) * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)P.A, (short)0, (int)a_ext, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)P.B, (short)0, (int)b_ext, 0x00020000);
  const int nk = P.K / BK;
#define SA(s) (smem + (s) * (TILE_T + TILE_BYTES))
#define SB(s) (SA(s) + TILE_T)
  auto dma_a = [&](char* lds, int bm, int k0) {
#pragma unroll
    for (int x = 0; x < FRT; ++x) {
      const int ins = wid * FRT + x;
      const int row = ins * 8 + (lane >> 3), c = (lane & 7) ^ (row & 7);
      const int voff = (int)(((long)(bm + row) * P.lda + k0 + c * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(lds + ins * 1024), 16, voff, 0, 0, 0);
    }
  };
  auto coords = [&](int lin, int& bm, int& bn) {
    int z, tm, tn;
    tile_coords(lin, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
    bm = tm * BMT;
    bn = tn * BN;
  };
  int bm, bn;
  coords(blockIdx.x, bm, bn);
  dma_a(SA(1), bm, 0);
  dma_tile<true>(rb, SB(1), P.ldb, bn, 0, wid, lane);
  bool counted = false;   // the previous tile's epilogue stores are the only VMEM ops after the prefetch
  for (int lin = blockIdx.x; lin < total; lin += gridDim.x) {
    f32x4 acc[FRT][4];
#pragma unroll
    for (int i = 0; i < FRT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      if (kt == 0 && counted) wait_vm<2 * FRT>();   // the prefetch, not the stores behind it
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      const int cur = (kt + 1) & 1;
      if (kt + 1 < nk) {
        dma_a(SA(cur ^ 1), bm, (kt + 1) * BK);
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
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FRT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb2[kk][j], fa2[kk][i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    __syncthreads();   // every wave past its last operand read of this tile
    const int cbm = bm, cbn = bn;
    const int nxt = lin + (int)gridDim.x;
    if (nxt < total) {
      coords(nxt, bm, bn);
      dma_a(SA(1), bm, 0);
      dma_tile<true>(rb, SB(1), P.ldb, bn, 0, wid, lane);
    }
    // full tile, 16-B fast path: exactly one store per epilogue row pass (2 FRT per wave)
    counted = cbm + BMT <= P.M && cbn + BN <= P.N && P.vec16;
    constexpr int WR = 16 * FRT;
#pragma unroll
    for (int ps = 0; ps < FRT / 2; ++ps) {
      if (ps) __syncthreads();
      staged_epilogue<EPI, 2, 32 * 64>(P, smem, reinterpret_cast<const f32x4(&)[2][4]>(acc[2 * ps]),
                                       cbm + WR * wm + 32 * ps - 64 * wm, cbn, wm, wn, wid, lane, P.C, P.aux);
    }
  }
#undef SA
#undef SB
}

template <int FRT>
int launch_pf_t(int epi, const GemmP& P, hipStream_t s) {
  constexpr int BMT = 32 * FRT;
  const int tm = (P.M + BMT - 1) / BMT, tn = (P.N + 127) / 128, total = tm * tn;
  const int grid = total < 512 ? total : 512;
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_pf_kernel<E, FRT>), dim3(grid), dim3(NT), 0, s, P, tm, tn, total); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_RELU_DROP_BWD)
#undef CASE
    default: return 1;
  }
  return hipGetLastError() != hipSuccess;
}
int launch_pf(int epi, int bm, const GemmP& P, hipStream_t s) {
  if (bm == 192) return launch_pf_t<6>(epi, P, s);
  if (bm == 128) return launch_pf_t<4>(epi, P, s);
  return 1;
}
}  // namespace
}  // namespace mmst
