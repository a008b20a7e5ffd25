// Wide-tile NT GEMM for gfx950: C[M, N] = epilogue(A[M, K] . B[N, K]^T), both operands
// K-contiguous (the step's forward projections and, through the W^T images, its dgrads).
//
// Why wide: with 128-row x 128-column tiles at two blocks per CU every CU stages 64 FLOP per
// operand byte through its load path (LDS-DMA issue, L2 -> LDS), and that intake, not the matrix
// core, paced the step's GEMMs (round-4 ablation: the MFMA loop alone 1744 TF, with its DMA
// 997 TF).  One block per CU on a BM x 256 tile stages 85-128 FLOP per byte.
//
// Geometry: 512 threads = 8 waves in two groups of 4 (g = wave >> 2); group g owns tile rows
// [g BM/2, (g+1) BM/2), wave (g, c) the 16 FM x 64 sub-tile at column 64 c (FM x 4 fragments of
// v_mfma_f32_16x16x32_f16).  BM = 32 FM, BN = 256.  K is walked in slots of 32 KS (KS = 1 or 2)
// through an R-slot LDS ring filled by buffer_load ... lds (16 B per lane, lane-linear images,
// XOR swizzle on the global source address, read back with ds_read_b128 as gemm.hip's BK = 32 /
// BK = 64 images).
//
// Schedule (ping-pong): each slot is two segments per wave — the wave's row halves (KS = 1) or
// k halves (KS = 2) — and every segment is a load phase (fragment reads, DMA issue) followed by an
// MFMA phase (16 MFMAs), each closed by a block barrier.  Group 1 runs one barrier behind group 0,
// so on every SIMD (waves w and w + 4) one wave issues MFMAs while the other reads LDS and issues
// DMA.  Per slot t (group-relative, four barriers):
//     L0: read B (+ A half 0 | k half 0) of slot t     [group 1: issue part of slot t + R - 1]
//     M0: MFMAs                                        barrier
//     L1: read A half 1 (| B, A k half 1) of slot t    [group 0: issue its part of slot t + R - 1;
//                                                       group 1: rest of its part, wait slot t + 1]
//     M1: MFMAs                                        [group 0: wait slot t + 1]  barrier
// Group 0 DMAs the A image of a slot, group 1 the B image.  WAR: slot t's ring entry is refilled
// (with slot t + R) only after both groups' reads of slot t retired — group 1's last (L1 of slot
// t, retired at its M1) is one barrier before group 1's L0 of slot t + 1, and two before group 0's
// L1 of slot t + 1.  RAW: every wave waits (counted vmcnt: its later slots stay in flight) for its
// part of slot t + 1 before the barrier that precedes group 0's L0 of slot t + 1.
//
// Accumulation order per output element is the 128 x 128 kernel's (32-deep k-chunks ascending, the
// same MFMA with the same operands) and the epilogue is its staged_epilogue, so results are
// bit-identical to gemm_dma_kernel.
#pragma once
#include "../../multimodal-s2ut_amd/csrc/gemm_common.h"

namespace mmsw {
namespace {

// vmcnt(n) for a wave-uniform n in [0, 31]
MMS_DEV void wait_vm_n(int n) {
  switch (n) {
#define WVN_CASE(k) case k: wait_vm<k>(); break;
    WVN_CASE(1) WVN_CASE(2) WVN_CASE(3) WVN_CASE(4) WVN_CASE(5) WVN_CASE(6) WVN_CASE(7) WVN_CASE(8) WVN_CASE(9) WVN_CASE(10)
    WVN_CASE(11) WVN_CASE(12) WVN_CASE(13) WVN_CASE(14) WVN_CASE(15) WVN_CASE(16) WVN_CASE(17) WVN_CASE(18) WVN_CASE(19)
    WVN_CASE(20) WVN_CASE(21) WVN_CASE(22) WVN_CASE(23) WVN_CASE(24) WVN_CASE(25) WVN_CASE(26) WVN_CASE(27) WVN_CASE(28)
    WVN_CASE(29) WVN_CASE(30) WVN_CASE(31)
#undef WVN_CASE
    default: wait_vm<0>(); break;
  }
}


constexpr int W_NT = 512;
// lab diagnostic: per block {s_memtime, s_memrealtime} at entry and exit (clock under load)
__device__ unsigned long long* g_w_clk = nullptr;

template <int FM, int KS, int R>
struct WGeo {
  static constexpr int BM = 32 * FM, BN = 256, BK = 32 * KS;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int SLOT = A_BYTES + B_BYTES;
  static constexpr int PA = A_BYTES / 1024 / 4;   // A pieces (1 KiB wave-instructions) per group-0 wave
  static constexpr int PB = B_BYTES / 1024 / 4;   // B pieces per group-1 wave
  static constexpr int PB0 = PB / 2;              // ... issued in group 1's first load phase
  static constexpr int RING = R * SLOT;
  static constexpr int LDS = RING > 8 * 16384 ? RING : 8 * 16384;   // the epilogue stages 16 KiB per wave
  static_assert(A_BYTES % 4096 == 0 && B_BYTES % 4096 == 0, "pieces per wave");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(R >= 3, "ring too shallow");
};

MMS_DEV void w_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// vmcnt(c * P) for c in [0, CMAX]
template <int P, int CMAX>
MMS_DEV void w_wait(int c) {
  if (CMAX >= 3 && c >= 3) wait_vm<(CMAX >= 3 ? 3 * P : 0)>();
  else if (CMAX >= 2 && c >= 2) wait_vm<(CMAX >= 2 ? 2 * P : 0)>();
  else if (c >= 1) wait_vm<P>();
  else wait_vm<0>();
}

// one 1 KiB piece of a K-contiguous slot image (rows of 32 KS k): BK = 32 -> 16 rows x 64 B
// (read_frag32's swizzle), BK = 64 -> 8 rows x 128 B (read_frag's swizzle)
template <int KS>
MMS_DEV void w_dma(__amdgpu_buffer_rsrc_t rs, char* img, long ld, int row0, int k0, int ins, int lane) {
  int voff;
  if (KS == 1) {
    const int row = ins * 16 + (lane >> 2);
    const int c = (lane & 3) ^ swz32(row);
    voff = (int)(((long)(row0 + row) * ld + k0 + c * 8) * 2);
  } else {
    const int row = ins * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (row & 7);
    voff = (int)(((long)(row0 + row) * ld + k0 + c * 8) * 2);
  }
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + ins * 1024), 16, voff, 0, 0, 0);
}

template <int KS>
MMS_DEV h16x8 w_frag(const char* img, int sub, int kk, int lane) {
  if (KS == 1) return read_frag32<true>(img, sub, lane);
  return read_frag<true>(img, sub, kk, lane);
}

// ABL (lab ablations, garbage results): 1 no operand DMA, 2 no LDS fragment reads, 4 no MFMA
// SCHED: 0 = the slot's DMA in one burst per group (group 1 in L0 + L1, group 0 in L1), slot t + R - 1
//        issued in iteration t; 1 = balanced, half of each group's part of slot t + R - 2 at the top of
//        each of its load phases; 2 = the same halves behind each MFMA phase's MFMAs
template <int EPI, int FM, int KS, int R, bool NOEPI = false, int ABL = 0, int SCHED = 1>
__global__ void __launch_bounds__(W_NT, 2) gemm_wide_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  using G = WGeo<FM, KS, R>;
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  (void)z;
  const int bm = tm * G::BM, bn = tn * G::BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wid >> 2, wc = wid & 3;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.A, (short)0, (int)(((long)(P.M - 1) * P.lda + P.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.B, (short)0, (int)(((long)(P.N - 1) * P.ldb + P.K) * 2), 0x00020000);
  const int nk = P.K / G::BK;   // host: K % BK == 0, K > 0
  constexpr int FH = KS == 1 ? FM / 2 : FM;   // A fragments read per load phase
  constexpr bool PR = PRIO && EPI != MMS_EPI_F32;
  // pieces of this wave's part of a slot issued in the first half (the rest in the second)
  constexpr int PA0 = (G::PA + 1) / 2, PB0 = (G::PB + 1) / 2;
  // slots ahead of the one being read that are in flight (DMA target = t + AHEAD in iteration t)
  constexpr int AHEAD = SCHED == 0 ? R - 1 : R - 2;

  f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto slot_ptr = [&](int t) { return smem + (t % R) * G::SLOT; };
  // this wave's pieces [lo, hi) of its part of slot t: group 0 the A image, group 1 the B image
  auto issue = [&](int t, int lo_a, int hi_a, int lo_b, int hi_b) {
    if (ABL & 1) return;
    char* s = slot_ptr(t);
    if (g == 0) {
#pragma unroll
      for (int x = 0; x < G::PA; ++x)
        if (x >= lo_a && x < hi_a) w_dma<KS>(ra, s, P.lda, bm, t * G::BK, wc * G::PA + x, lane);
    } else {
#pragma unroll
      for (int x = 0; x < G::PB; ++x)
        if (x >= lo_b && x < hi_b) w_dma<KS>(rb, s + G::A_BYTES, P.ldb, bn, t * G::BK, wc * G::PB + x, lane);
    }
  };
  // this wave's part of slot u has landed, its parts up to slot `issued` being out
  auto wait_slot = [&](int u, int issued) {
    const int c = min(issued, nk - 1) - u;
    if (g == 0) w_wait<G::PA, AHEAD - 1>(c);
    else w_wait<G::PB, AHEAD - 1>(c);
  };

#pragma unroll
  for (int t = 0; t < AHEAD; ++t)
    if (t < nk) issue(t, 0, G::PA, 0, G::PB);
  wait_slot(0, AHEAD - 1);
  w_barrier();
  if (g) w_barrier();   // the stagger
  const int arow = g * (G::BM / 2), bcol = wc * 64;
  for (int t = 0; t < nk; ++t) {
    const char* s = slot_ptr(t);
    const char* sb = s + G::A_BYTES;
    const int nxt = t + AHEAD;
    const bool more = nxt < nk;
    h16x8 fb[4], fa[FH];
    // ---- L0
    if (SCHED == 1 && more) issue(nxt, 0, PA0, 0, PB0);
    if (ABL & 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { fb[j] = h16x8{}; asm volatile("" : "+v"(fb[j])); }
#pragma unroll
      for (int i = 0; i < FH; ++i) { fa[i] = h16x8{}; asm volatile("" : "+v"(fa[i])); }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = w_frag<KS>(sb, bcol + j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < FH; ++i) fa[i] = w_frag<KS>(s, arow + i * 16, 0, lane);
    }
    if (SCHED == 0 && g == 1 && more) issue(nxt, 0, 0, 0, G::PB / 2);
    w_barrier();
    // ---- M0
    if (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FH; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (ABL & 4) asm volatile("" :: "v"(fb[j]), "v"(fa[i]));
        else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    if (PR) __builtin_amdgcn_s_setprio(0);
    if (SCHED == 2 && more) issue(nxt, 0, PA0, 0, PB0);
    w_barrier();
    // ---- L1
    if (SCHED == 1 && more) issue(nxt, PA0, G::PA, PB0, G::PB);
    if (ABL & 2) {
#pragma unroll
      for (int i = 0; i < FH; ++i) asm volatile("" : "+v"(fa[i]));
    } else if (KS == 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = w_frag<KS>(sb, bcol + j * 16, 1, lane);
#pragma unroll
      for (int i = 0; i < FH; ++i) fa[i] = w_frag<KS>(s, arow + i * 16, 1, lane);
    } else {
#pragma unroll
      for (int i = 0; i < FH; ++i) fa[i] = w_frag<KS>(s, arow + (FH + i) * 16, 0, lane);
    }
    if (SCHED == 0 && more) issue(nxt, 0, G::PA, G::PB / 2, G::PB);
    if (SCHED != 2 && g == 1 && t + 1 < nk) wait_slot(t + 1, nxt);
    if (SCHED == 2 && g == 1 && t + 1 < nk) {
      // slot nxt is half issued (M0): younger than slot t + 1 are the whole slots t + 2 .. nxt - 1
      // and the first PB0 pieces of nxt
      const int full = min(nxt - 1, nk - 1) - (t + 1);
      wait_vm_n(full * G::PB + (more ? PB0 : 0));
    }
    w_barrier();
    // ---- M1
    if (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FH; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        constexpr int o = KS == 1 ? FH : 0;
        if (ABL & 4) asm volatile("" :: "v"(fb[j]), "v"(fa[i]));
        else acc[o + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[o + i][j], 0, 0, 0);
      }
    if (PR) __builtin_amdgcn_s_setprio(0);
    if (SCHED == 2 && more) issue(nxt, PA0, G::PA, PB0, G::PB);
    if (g == 0 && t + 1 < nk) wait_slot(t + 1, nxt);
    w_barrier();
  }
  if (!g) w_barrier();   // matches group 1's stagger: every wave is past its last LDS read and DMA wait
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  if (NOEPI) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  char* Cz = reinterpret_cast<char*>(P.C);
  constexpr int F1 = FM < 4 ? FM : 4;
  staged_epilogue<EPI, F1>(P, smem, reinterpret_cast<const f32x4(&)[F1][4]>(acc[0]), bm + arow, bn + bcol, 0, 0,
                           wid, lane, Cz, P.aux);
  if constexpr (FM > 4) {
    __syncthreads();
    staged_epilogue<EPI, FM - 4>(P, smem, reinterpret_cast<const f32x4(&)[FM - 4][4]>(acc[4]), bm + arow + 64,
                                 bn + bcol, 0, 0, wid, lane, Cz, P.aux);
  }
  stamp_end(P.stamps, t_start);
}

template <int FM, int KS, int R, bool NOEPI, int ABL = 0, int SCHED = 1>
int launch_wide_t(int epi, const GemmP& P, hipStream_t s) {
  using G = WGeo<FM, KS, R>;
  const int tm = (P.M + G::BM - 1) / G::BM, tn = (P.N + G::BN - 1) / G::BN;
  const int total = tm * tn;
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_wide_kernel<E, FM, KS, R, NOEPI, ABL, SCHED>), dim3(total), dim3(W_NT), 0, s, P, tm, tn, total); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_RELU_DROP_BWD)
#undef CASE
    default: return 1;
  }
  return hipGetLastError() != hipSuccess;
}

// ------------------------------------------------------------------------------------------
// 64-deep slots (full 128-B rows per DMA piece: the 32-deep images above fetch every operand line
// in two half-line requests, and measured ~35 % less LDS-DMA throughput), a 2-slot ring, and every
// fragment of a slot read into registers in the slot's first two load phases so its ring entry is
// free (for slot t + 2) half-way through the slot.  Per slot t, four segments per wave:
//     L0: read B (both k halves) + A rows lo (both)   M0: rows lo, k 0-31
//     L1: read A rows hi (both)                        M1: rows lo, k 32-63
//     L2: [group 1: B part of slot t+2, half]          M2: rows hi, k 0-31  [group 0: A part, half]
//     L3: [group 1: rest; group 0: rest;               M3: rows hi, k 32-63 [group 0: wait t+1]
//          group 1: wait slot t+1]
// Reads of slot t retire by group 1's M1 (one barrier before group 1's L2): its entry is free.
// ------------------------------------------------------------------------------------------
template <int EPI, int FM, bool NOEPI = false, int ABL = 0>
__global__ void __launch_bounds__(W_NT, 2) gemm_wide2_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  constexpr int BM = 32 * FM, BN = 256, BKS = 64;
  constexpr int A_BYTES = BM * BKS * 2, B_BYTES = BN * BKS * 2, SLOT = A_BYTES + B_BYTES;
  constexpr int PA = A_BYTES / 4096, PB = B_BYTES / 4096;   // pieces per wave per slot
  constexpr int LDS = 2 * SLOT > 8 * 16384 ? 2 * SLOT : 8 * 16384;
  constexpr int FH = FM / 2;
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  unsigned long long* clk = g_w_clk;
  unsigned long long c0 = 0, r0 = 0;
  if (clk) { c0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  (void)z;
  const int bm = tm * BM, bn = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wid >> 2, wc = wid & 3;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.A, (short)0, (int)(((long)(P.M - 1) * P.lda + P.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.B, (short)0, (int)(((long)(P.N - 1) * P.ldb + P.K) * 2), 0x00020000);
  const int nk = P.K / BKS;
  constexpr bool PR = PRIO && EPI != MMS_EPI_F32;
  f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto slot_ptr = [&](int t) { return smem + (t & 1) * SLOT; };
  auto issue = [&](int t, int lo, int hi) {
    if (ABL & 1) return;
    char* s = slot_ptr(t);
    if (g == 0) {
#pragma unroll
      for (int x = 0; x < PA; ++x)
        if (x >= lo && x < hi) w_dma<2>(ra, s, P.lda, bm, t * BKS, wc * PA + x, lane);
    } else {
#pragma unroll
      for (int x = 0; x < PB; ++x)
        if (x >= lo && x < hi) w_dma<2>(rb, s + A_BYTES, P.ldb, bn, t * BKS, wc * PB + x, lane);
    }
  };
  constexpr int PW = PA > PB ? PA : PB;
  const int pw = g == 0 ? PA : PB;   // this wave's pieces per slot
  (void)PW;
  issue(0, 0, PW);
  if (nk > 1) issue(1, 0, PW);
  wait_vm_n(nk > 1 ? pw : 0);
  w_barrier();
  if (g) w_barrier();
  const int arow = g * (BM / 2), bcol = wc * 64;
  auto mfma_seg = [&](const h16x8 (&fa)[FH], const h16x8 (&fb)[4], int o) {
    if (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FH; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (ABL & 4) asm volatile("" :: "v"(fb[j]), "v"(fa[i]));
        else acc[o + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[o + i][j], 0, 0, 0);
      }
    if (PR) __builtin_amdgcn_s_setprio(0);
  };
  const int ph = pw / 2;
  for (int t = 0; t < nk; ++t) {
    const char* s = slot_ptr(t);
    const char* sb = s + A_BYTES;
    const bool more = t + 2 < nk;
    h16x8 fb0[4], fb1[4], fl0[FH], fl1[FH], fh0[FH], fh1[FH];
    // L0
#pragma unroll
    for (int j = 0; j < 4; ++j) { fb0[j] = read_frag<true>(sb, bcol + j * 16, 0, lane); fb1[j] = read_frag<true>(sb, bcol + j * 16, 1, lane); }
#pragma unroll
    for (int i = 0; i < FH; ++i) { fl0[i] = read_frag<true>(s, arow + i * 16, 0, lane); fl1[i] = read_frag<true>(s, arow + i * 16, 1, lane); }
    w_barrier();
    mfma_seg(fl0, fb0, 0);   // M0
    w_barrier();
    // L1
#pragma unroll
    for (int i = 0; i < FH; ++i) { fh0[i] = read_frag<true>(s, arow + (FH + i) * 16, 0, lane); fh1[i] = read_frag<true>(s, arow + (FH + i) * 16, 1, lane); }
    w_barrier();
    // every read of slot t retires here (WAR: group 1's L2, two barriers on, refills the entry)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfma_seg(fl1, fb1, 0);   // M1
    w_barrier();
    // L2
    if (g == 1 && more) issue(t + 2, 0, ph);
    w_barrier();
    mfma_seg(fh0, fb0, FH);   // M2
    if (g == 0 && more) issue(t + 2, 0, ph);
    w_barrier();
    // L3
    if (more) issue(t + 2, ph, pw);
    if (g == 1 && t + 1 < nk) wait_vm_n(more ? pw : 0);
    w_barrier();
    mfma_seg(fh1, fb1, FH);   // M3
    if (g == 0 && t + 1 < nk) wait_vm_n(more ? pw : 0);
    w_barrier();
  }
  if (!g) w_barrier();
  if (clk && threadIdx.x == 0) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    typedef unsigned long long u64x4_ __attribute__((ext_vector_type(4)));
    *reinterpret_cast<u64x4_*>(clk + 4 * (long)blockIdx.x) = u64x4_{c0, r0, c1, r1};
  }
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  if (NOEPI) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  char* Cz = reinterpret_cast<char*>(P.C);
  constexpr int F1 = FM < 4 ? FM : 4;
  staged_epilogue<EPI, F1>(P, smem, reinterpret_cast<const f32x4(&)[F1][4]>(acc[0]), bm + arow, bn + bcol, 0, 0,
                           wid, lane, Cz, P.aux);
  if constexpr (FM > 4) {
    __syncthreads();
    staged_epilogue<EPI, FM - 4>(P, smem, reinterpret_cast<const f32x4(&)[FM - 4][4]>(acc[4]), bm + arow + 64,
                                 bn + bcol, 0, 0, wid, lane, Cz, P.aux);
  }
  stamp_end(P.stamps, t_start);
}

template <int FM, bool NOEPI, int ABL = 0>
int launch_wide2_t(int epi, const GemmP& P, hipStream_t s) {
  constexpr int BM = 32 * FM;
  const int tm = (P.M + BM - 1) / BM, tn = (P.N + 255) / 256;
  const int total = tm * tn;
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_wide2_kernel<E, FM, NOEPI, ABL>), dim3(total), dim3(W_NT), 0, s, P, tm, tn, total); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_RELU_DROP_BWD)
#undef CASE
    default: return 1;
  }
  return hipGetLastError() != hipSuccess;
}

// ------------------------------------------------------------------------------------------
// Operand ring: a 5-entry ring of 32 KiB operand images in the order A(0) B(0) A(1) B(1) ...
// (image u lives in entry u % 5; A images of 32 FM rows, B images of 256 rows, 64 k deep, full
// 128-B rows per DMA piece).  Two and a half k-tiles of buffering: while k-tile t computes, A(t+1),
// B(t+1), A(t+2) land and, once k-tile t's reads retire (group 1's M1), B(t+2) and A(t+3) are
// issued into the entries of A(t) and B(t).  Waits: group 0 (A) at the end of its M3 for A(t+1)
// with A(t+2), A(t+3) in flight; group 1 (B) at the end of its L3 for B(t+1) with B(t+2) in flight.
// ------------------------------------------------------------------------------------------
template <int EPI, int FM, bool NOEPI = false, int ABL = 0>
__global__ void __launch_bounds__(W_NT, 2) gemm_wide3_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  constexpr int BM = 32 * FM, BN = 256, BKS = 64, ENT = 32768;
  constexpr int PA = BM * BKS * 2 / 4096, PB = BN * BKS * 2 / 4096;   // pieces per wave per image
  constexpr int FH = FM / 2;
  static_assert(BM <= 256, "A image must fit an entry");
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  __shared__ __attribute__((aligned(16))) char smem[5 * ENT];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  (void)z;
  const int bm = tm * BM, bn = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wid >> 2, wc = wid & 3;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.A, (short)0, (int)(((long)(P.M - 1) * P.lda + P.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.B, (short)0, (int)(((long)(P.N - 1) * P.ldb + P.K) * 2), 0x00020000);
  const int nk = P.K / BKS;
  constexpr bool PR = PRIO && EPI != MMS_EPI_F32;
  f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto img_a = [&](int t) { return smem + ((2 * t) % 5) * ENT; };
  auto img_b = [&](int t) { return smem + ((2 * t + 1) % 5) * ENT; };
  // group 0 issues A images, group 1 B images; pieces [lo, hi) of its part
  auto issue_a = [&](int t, int lo, int hi) {
    if (ABL & 1) return;
    char* s = img_a(t);
#pragma unroll
    for (int x = 0; x < PA; ++x)
      if (x >= lo && x < hi) w_dma<2>(ra, s, P.lda, bm, t * BKS, wc * PA + x, lane);
  };
  auto issue_b = [&](int t, int lo, int hi) {
    if (ABL & 1) return;
    char* s = img_b(t);
#pragma unroll
    for (int x = 0; x < PB; ++x)
      if (x >= lo && x < hi) w_dma<2>(rb, s, P.ldb, bn, t * BKS, wc * PB + x, lane);
  };
  if (g == 0) {
    issue_a(0, 0, PA);
    if (nk > 1) issue_a(1, 0, PA);
    if (nk > 2) issue_a(2, 0, PA);
    wait_vm_n(PA * (min(nk, 3) - 1));
  } else {
    issue_b(0, 0, PB);
    if (nk > 1) issue_b(1, 0, PB);
    wait_vm_n(nk > 1 ? PB : 0);
  }
  w_barrier();
  if (g) w_barrier();
  const int arow = g * (BM / 2), bcol = wc * 64;
  auto mfma_seg = [&](const h16x8 (&fa)[FH], const h16x8 (&fb)[4], int o) {
    if (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FH; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (ABL & 4) asm volatile("" :: "v"(fb[j]), "v"(fa[i]));
        else acc[o + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[o + i][j], 0, 0, 0);
      }
    if (PR) __builtin_amdgcn_s_setprio(0);
  };
  constexpr int HA = PA / 2, HB = PB / 2;
  for (int t = 0; t < nk; ++t) {
    const char* sa = img_a(t);
    const char* sb = img_b(t);
    h16x8 fb0[4], fb1[4], fl0[FH], fl1[FH], fh0[FH], fh1[FH];
#pragma unroll
    for (int j = 0; j < 4; ++j) { fb0[j] = read_frag<true>(sb, bcol + j * 16, 0, lane); fb1[j] = read_frag<true>(sb, bcol + j * 16, 1, lane); }
#pragma unroll
    for (int i = 0; i < FH; ++i) { fl0[i] = read_frag<true>(sa, arow + i * 16, 0, lane); fl1[i] = read_frag<true>(sa, arow + i * 16, 1, lane); }
    w_barrier();
    mfma_seg(fl0, fb0, 0);   // M0
    w_barrier();
#pragma unroll
    for (int i = 0; i < FH; ++i) { fh0[i] = read_frag<true>(sa, arow + (FH + i) * 16, 0, lane); fh1[i] = read_frag<true>(sa, arow + (FH + i) * 16, 1, lane); }
    w_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // every read of k-tile t retires here
    mfma_seg(fl1, fb1, 0);   // M1
    w_barrier();
    if (g == 1 && t + 2 < nk) issue_b(t + 2, 0, HB);   // L2
    w_barrier();
    mfma_seg(fh0, fb0, FH);   // M2
    if (g == 0 && t + 3 < nk) issue_a(t + 3, 0, HA);
    w_barrier();
    if (g == 1 && t + 2 < nk) issue_b(t + 2, HB, PB);   // L3
    if (g == 0 && t + 3 < nk) issue_a(t + 3, HA, PA);
    if (g == 1 && t + 1 < nk) wait_vm_n(t + 2 < nk ? PB : 0);
    w_barrier();
    mfma_seg(fh1, fb1, FH);   // M3
    if (g == 0 && t + 1 < nk) wait_vm_n(PA * ((t + 2 < nk ? 1 : 0) + (t + 3 < nk ? 1 : 0)));
    w_barrier();
  }
  if (!g) w_barrier();
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  if (NOEPI) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  char* Cz = reinterpret_cast<char*>(P.C);
  constexpr int F1 = FM < 4 ? FM : 4;
  staged_epilogue<EPI, F1>(P, smem, reinterpret_cast<const f32x4(&)[F1][4]>(acc[0]), bm + arow, bn + bcol, 0, 0,
                           wid, lane, Cz, P.aux);
  if constexpr (FM > 4) {
    __syncthreads();
    staged_epilogue<EPI, FM - 4>(P, smem, reinterpret_cast<const f32x4(&)[FM - 4][4]>(acc[4]), bm + arow + 64,
                                 bn + bcol, 0, 0, wid, lane, Cz, P.aux);
  }
  stamp_end(P.stamps, t_start);
}

template <int FM, bool NOEPI, int ABL = 0>
int launch_wide3_t(int epi, const GemmP& P, hipStream_t s) {
  constexpr int BM = 32 * FM;
  const int tm = (P.M + BM - 1) / BM, tn = (P.N + 255) / 256;
  const int total = tm * tn;
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_wide3_kernel<E, FM, NOEPI, ABL>), dim3(total), dim3(W_NT), 0, s, P, tm, tn, total); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_RELU_DROP_BWD)
#undef CASE
    default: return 1;
  }
  return hipGetLastError() != hipSuccess;
}

// lab dispatch: variant = schedule / ring / ablation code
int launch_wide(int epi, int bm, int variant, GemmP P, hipStream_t s, bool noepi) {
  P.group_m = 8;
  if (bm > 3000) {   // operand ring
    const int h = bm - 3000;
    if (noepi) {
      if (h == 256) return variant == 1 ? launch_wide3_t<8, true, 1>(epi, P, s) : variant == 4 ? launch_wide3_t<8, true, 4>(epi, P, s) : launch_wide3_t<8, true, 0>(epi, P, s);
      if (h == 192) return launch_wide3_t<6, true, 0>(epi, P, s);
      if (h == 128) return launch_wide3_t<4, true, 0>(epi, P, s);
      return 1;
    }
    if (h == 256) return launch_wide3_t<8, false>(epi, P, s);
    if (h == 192) return launch_wide3_t<6, false>(epi, P, s);
    if (h == 128) return launch_wide3_t<4, false>(epi, P, s);
    return 1;
  }
  if (bm > 1000) {   // 64-deep slots, 2-slot ring, early reads (variant: ablation bits when noepi)
    const int h = bm - 2000;
    if (noepi) {
      if (h == 256) return variant == 1 ? launch_wide2_t<8, true, 1>(epi, P, s) : variant == 4 ? launch_wide2_t<8, true, 4>(epi, P, s) : launch_wide2_t<8, true, 0>(epi, P, s);
      if (h == 192) return launch_wide2_t<6, true, 0>(epi, P, s);
      if (h == 128) return launch_wide2_t<4, true, 0>(epi, P, s);
      return 1;
    }
    if (h == 256) return launch_wide2_t<8, false>(epi, P, s);
    if (h == 192) return launch_wide2_t<6, false>(epi, P, s);
    if (h == 128) return launch_wide2_t<4, false>(epi, P, s);
    return 1;
  }
  if (bm == 256) {
    if (noepi) {
      switch (variant) {
        case 0: return launch_wide_t<8, 1, 4, true, 0, 0>(epi, P, s);   // old schedule
        case 1: return launch_wide_t<8, 1, 4, true, 0, 1>(epi, P, s);
        case 2: return launch_wide_t<8, 1, 5, true, 0, 1>(epi, P, s);
        case 3: return launch_wide_t<8, 1, 4, true, 0, 2>(epi, P, s);
        case 4: return launch_wide_t<8, 1, 5, true, 0, 2>(epi, P, s);
        case 5: return launch_wide_t<8, 1, 5, true, 1, 1>(epi, P, s);   // no DMA
        case 6: return launch_wide_t<8, 1, 5, true, 4, 1>(epi, P, s);   // no MFMA
        default: return 1;
      }
    }
    switch (variant) {
      case 0: return launch_wide_t<8, 1, 4, false, 0, 0>(epi, P, s);
      case 1: return launch_wide_t<8, 1, 5, false, 0, 1>(epi, P, s);
      case 2: return launch_wide_t<8, 1, 5, false, 0, 2>(epi, P, s);
      default: return 1;
    }
  }
  if (bm == 128) {
    if (noepi) return variant == 1 ? launch_wide_t<4, 2, 3, true, 0, 1>(epi, P, s) : launch_wide_t<4, 2, 3, true, 0, 0>(epi, P, s);
    return variant == 1 ? launch_wide_t<4, 2, 3, false, 0, 1>(epi, P, s) : launch_wide_t<4, 2, 3, false, 0, 0>(epi, P, s);
  }
  return 1;
}

}  // namespace
}  // namespace mmsw
