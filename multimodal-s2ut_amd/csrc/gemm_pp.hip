// Ping-pong 256-column NT GEMM for gfx950: C[M, N] = epilogue(A[M, K] . B[N, K]^T), both operands
// K-contiguous (the step's forward projections and, through the W^T images, its dgrads).
//
// Tile BM x 256 (BM = 128 / 192 / 256, picked per shape so the grid fills the 256 CUs in whole
// rounds), one 512-thread block per CU: 8 waves as 2 row groups x 4 column waves, wave tile
// (BM/2) x 64 = (BM/32) x 4 fragments of v_mfma_f32_16x16x32_f16.  K is walked in 32-deep slots
// through an R-slot LDS ring filled by buffer_load ... lds (16 B per lane, lane-linear image, XOR
// swizzle on the global source address, read back with ds_read_b128 exactly as the BK = 32 images
// of gemm.hip).
//
// The two row groups run one barrier apart (group 1 passes one extra barrier first), so at every
// barrier one group starts its MFMA block while the other starts reading its next slot's fragments
// and issuing DMA: on each SIMD (waves w and w + 4) one wave feeds the matrix core while the other
// waits on LDS / memory.  Per slot s, barrier-delimited segments:
//     group 0:  [read s]  |  [MFMA s, issue A(s+L), wait A(s+1)]        |
//     group 1:            |  [read s, issue B(s+L), wait B(s+1)]  |  [MFMA s]
// Group 0 DMAs every slot's A image (BM/16 wave-instructions over its 4 waves), group 1 its B image
// (16).  Each wave waits only for its own DMA with a counted vmcnt (L - 1 later slots stay in
// flight) before the barrier that precedes the first read of that slot (RAW).  Slot s + L goes
// into the ring position of slot s - 1 (L = R - 1), whose reads both groups retired (lgkmcnt)
// before the barrier the issuing wave passed last (WAR): group 1's read of slot s - 1 ended one
// segment before group 0's MFMA segment of slot s, group 0's one segment before group 1's read
// segment of slot s.
//
// Accumulation order per output element is the 128x128 kernel's (32-deep k-chunks ascending, the
// same MFMA with the same operands), and the epilogue is its staged_epilogue: results are
// bit-identical to gemm_dma_kernel (tests/test_gpu_gemm_splitk.py::test_pp_gemm_bit_identical).
#include "gemm_common.h"

namespace {

constexpr int PP_BN = 256, PP_NT = 512, PP_BK = 32;

template <int BM>
struct PPGeo {
  static constexpr int FA = BM / 32;                  // A fragments per wave per slot
  static constexpr int A_BYTES = BM * PP_BK * 2;      // slot images: A [BM][32], B [256][32] fp16
  static constexpr int B_BYTES = PP_BN * PP_BK * 2;
  static constexpr int SLOT = A_BYTES + B_BYTES;
  static constexpr int R0 = (160 * 1024) / SLOT;
  static constexpr int R = R0 > 6 ? 6 : R0;           // ring slots (256: 5 x 32 KiB, 192: 5 x 28, 128: 6 x 24)
  static constexpr int L = R - 1;                     // slots issued ahead of the one being read
  static constexpr int NI_A = BM / 64;                // A wave-instructions per group-0 wave per slot
  static constexpr int NI_B = 4;                      // B: 16 per slot over the 4 group-1 waves
  static_assert(R * SLOT >= 8 * 64 * 64 * 4, "the staged epilogue needs 16 KiB per wave");
  static_assert(L >= 2, "ring too shallow");
};

#ifdef MMS_PP_DIAG
// diagnostic build (scripts/build_ab.sh NAME gemm_pp.hip -DMMS_PP_DIAG): waves 0 and 4 of every block
// sum s_memtime cycles per loop segment: [0] read + issue (+ group 1's DMA wait), [1] barrier 1,
// [2] MFMA issue (+ group 0's DMA wait), [3] barrier 2, [4] slots timed, [5] whole loop
__device__ unsigned long long* g_pp_diag = nullptr;
extern "C" int mms2ut_pp_diag_bind(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pp_diag), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
#define PP_T(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (s >= 2) dsum[i] += t_ - t_prev; t_prev = t_; } while (0)
#else
#define PP_T(i) do { } while (0)
#endif

MMS_DEV void pp_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// vmcnt(c * NI) for c in [0, CMAX]
template <int NI, int CMAX>
MMS_DEV void wait_parts(int c) {
  if (CMAX >= 4 && c >= 4) wait_vm<(CMAX >= 4 ? 4 * NI : 0)>();
  else if (CMAX >= 3 && c == 3) wait_vm<(CMAX >= 3 ? 3 * NI : 0)>();
  else if (c == 2) wait_vm<2 * NI>();
  else if (c == 1) wait_vm<NI>();
  else wait_vm<0>();
}

// one 16-row x 32-k wave-instruction of a slot image: lane l fills row (l >> 2), 16-B chunk l & 3,
// with the global chunk (l & 3) ^ swz32(row) (read_frag32's swizzle)
MMS_DEV void pp_dma(__amdgpu_buffer_rsrc_t rs, char* img, long ld, int row0, int k0, int ins, int lane) {
#ifdef MMS_PP_L2HOT   // ablation build: every block streams the same 64 KiB (L2-resident; garbage results)
  row0 = 0;
  k0 &= 127;
#endif
  const int row = ins * 16 + (lane >> 2);
  const int c = (lane & 3) ^ swz32(row);
  const int voff = (int)(((long)(row0 + row) * ld + k0 + c * 8) * 2);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + ins * 1024), 16, voff, 0, 0, 0);
}

template <int EPI, int BM>
__global__ void __launch_bounds__(PP_NT, 2) gemm_pp_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  using G = PPGeo<BM>;
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  __shared__ __attribute__((aligned(16))) char smem[G::R * G::SLOT];
  int z, tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
  const int bm = tm * BM, bn = tn * PP_BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const bool g1 = wr != 0;
  // whole-operand descriptors; rows past M / N read as zero through the range check
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.A, (short)0, (int)(((long)(P.M - 1) * P.lda + P.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.B, (short)0, (int)(((long)(P.N - 1) * P.ldb + P.K) * 2), 0x00020000);
  const int nk = P.K / PP_BK;   // host: K % 32 == 0, K > 0

  f32x4 acc[G::FA][4];
#pragma unroll
  for (int i = 0; i < G::FA; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this wave's share of slot t's DMA: group 0 the A image, group 1 the B image
  auto issue = [&](int t) {
#ifdef MMS_PP_NODMA   // ablation build: no operand traffic (garbage results)
    return;
#endif
    char* slot = smem + (t % G::R) * G::SLOT;
    if (!g1) {
#pragma unroll
      for (int i = 0; i < G::NI_A; ++i) pp_dma(ra, slot, P.lda, bm, t * PP_BK, wid * G::NI_A + i, lane);
    } else {
#pragma unroll
      for (int i = 0; i < G::NI_B; ++i) pp_dma(rb, slot + G::A_BYTES, P.ldb, bn, t * PP_BK, (wid - 4) * G::NI_B + i, lane);
    }
  };
  // this wave's DMA of slot u has landed, given that its parts up to slot `issued` are out
  auto wait_slot = [&](int u, int issued) {
    const int c = min(issued, nk - 1) - u;   // later parts allowed in flight
    if (g1) wait_parts<G::NI_B, G::L - 1>(c);
    else wait_parts<G::NI_A, G::L - 1>(c);
  };

#pragma unroll
  for (int t = 0; t < G::L; ++t)
    if (t < nk) issue(t);
  wait_slot(0, G::L - 1);
  pp_barrier();
#ifndef MMS_PP_NOSTAGGER
  if (g1) pp_barrier();   // the stagger
#endif
  const int arow = wr * (BM / 2), bcol = wc * 64;
#ifdef MMS_PP_DIAG
  unsigned long long dsum[4] = {0, 0, 0, 0};
  unsigned long long t_prev = __builtin_amdgcn_s_memtime();
  const unsigned long long t_loop = t_prev;
#endif
  for (int s = 0; s < nk; ++s) {
    const char* slot = smem + (s % G::R) * G::SLOT;
    h16x8 fa[G::FA], fb[4];
#ifdef MMS_PP_NOREAD   // ablation build: fragments from registers, no LDS reads (garbage results)
#pragma unroll
    for (int j = 0; j < 4; ++j) { fb[j] = h16x8{}; asm volatile("" : "+v"(fb[j])); }
#pragma unroll
    for (int i = 0; i < G::FA; ++i) { fa[i] = h16x8{}; asm volatile("" : "+v"(fa[i])); }
    (void)slot;
#else
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = read_frag32<true>(slot + G::A_BYTES, bcol + j * 16, lane);
#pragma unroll
    for (int i = 0; i < G::FA; ++i) fa[i] = read_frag32<true>(slot, arow + i * 16, lane);
#endif
    if (g1 && s + G::L < nk) issue(s + G::L);
#ifdef MMS_PP_NOSTAGGER
    if (s + 1 < nk) wait_slot(s + 1, s + G::L);
#else
    if (g1 && s + 1 < nk) wait_slot(s + 1, s + G::L);
#endif
    PP_T(0);
    pp_barrier();
    PP_T(1);
#ifdef MMS_PP_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int i = 0; i < G::FA; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#ifdef MMS_PP_NOMFMA   // ablation build: keep the fragments live, no matrix work
        asm volatile("" :: "v"(fa[i]), "v"(fb[j]));
#else
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
#endif
      }
#ifdef MMS_PP_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    if (!g1 && s + G::L < nk) issue(s + G::L);
#ifndef MMS_PP_NOSTAGGER
    if (!g1 && s + 1 < nk) wait_slot(s + 1, s + G::L);
#endif
    PP_T(2);
    pp_barrier();
    PP_T(3);
  }
#ifdef MMS_PP_DIAG
  if (lane == 0 && (wid & 3) == 0 && g_pp_diag) {
    unsigned long long* o = g_pp_diag + ((long)blockIdx.x * 2 + wr) * 8;
    o[0] = dsum[0]; o[1] = dsum[1]; o[2] = dsum[2]; o[3] = dsum[3];
    o[4] = nk > 2 ? nk - 2 : 0; o[5] = __builtin_amdgcn_s_memtime() - t_loop;
  }
#endif
#ifndef MMS_PP_NOSTAGGER
  if (!g1) pp_barrier();   // matches group 1's stagger: every wave is past its last LDS read,
                           // and every DMA was waited for before its slot's first read
#endif
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  char* Cz = reinterpret_cast<char*>(P.C);
  const h16* auxz = P.aux;
  staged_epilogue<EPI, 4>(P, smem, reinterpret_cast<const f32x4(&)[4][4]>(acc[0]), bm + arow, bn + bcol,
                          0, 0, wid, lane, Cz, auxz);
  if constexpr (G::FA > 4) {
    __syncthreads();
    staged_epilogue<EPI, G::FA - 4>(P, smem, reinterpret_cast<const f32x4(&)[G::FA - 4][4]>(acc[4]),
                                    bm + arow + 64, bn + bcol, 0, 0, wid, lane, Cz, auxz);
  }
  stamp_end(P.stamps, t_start);
}

template <int BM>
int launch_bm(int epi, const GemmP& P, int tm, int tn, hipStream_t s) {
  const int total = tm * tn;
  dim3 grid(total), block(PP_NT);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_pp_kernel<E, BM>), grid, block, 0, s, P, tm, tn, total); break;
    MMS_EPI_CASES
#undef CASE
    default: mms::set_error("gemm_pp: bad epilogue %d", epi); return 1;
  }
  return mms::check_launch("gemm_pp");
}

}  // namespace

namespace mmsg {
int launch_pp(int epi, int bm, const GemmP& P, int tiles_m, int tiles_n, hipStream_t s) {
  switch (bm) {
    case 128: return launch_bm<128>(epi, P, tiles_m, tiles_n, s);
    case 192: return launch_bm<192>(epi, P, tiles_m, tiles_n, s);
    case 256: return launch_bm<256>(epi, P, tiles_m, tiles_n, s);
    default: mms::set_error("gemm_pp: bad tile height %d", bm); return 1;
  }
}
}  // namespace mmsg
