// Persistent 128x128 NT GEMM with a deferred epilogue (gfx950): C[M, N] = epilogue(A[M, K] . B[N, K]^T),
// both operands K-contiguous — the step's forward projections and (through the W^T images) dgrads.
//
// Why: in the one-tile-per-block kernel (gemm.hip gemm_dma_kernel) every tile of a round finishes
// its k-loop at about the same time, so the whole chip alternates between an MFMA phase (HBM idle)
// and an epilogue phase (every CU storing C, MFMAs idle).  On the short-K wide shapes (K = 768,
// N = 2304 / 3072) the epilogue was 35-40 % of the kernel (gemm.hip -DMMS_GEMM_NOEPI ablation,
// profiles/round4_gemm_ablation.txt).  Here each block (2 per CU, grid <= 512) walks a strided
// sequence of tiles of its XCD's range and runs tile i's epilogue INSIDE tile i+1's k-loop: two
// 16x16 accumulator fragments per k-step (math, dropout hash, 8-B stores), their aux / residual
// operands loaded one k-step ahead so the k-step's vmcnt(0) (which the 2-stage LDS-DMA ring takes
// anyway) has already retired them.  The last k-step of a tile DMAs the next tile's first stage,
// so the tile prologue's load latency is hidden as well.
//
// The k-loop is gemm_dma_kernel's (128x128x64 tiles, 4 waves of 64x64, 2-stage LDS-DMA ring,
// XOR-swizzled images, mfma_f32_16x16x32_f16 with (B, A) swapped) and the epilogue arithmetic is
// staged_epilogue's element for element, so results are bit-identical to gemm_dma_kernel
// (tests/test_gpu_gemm_splitk.py::test_dp_gemm_bit_identical).
#include <atomic>
#include <utility>

#include "gemm_common.h"

namespace {

constexpr int DP_PIECES = 2;   // accumulator fragments of the previous tile finished per k-step
constexpr int NP_ = 16 / DP_PIECES;   // k-steps of a tile that carry the previous tile's fragments

template <int EPI>
constexpr bool dp_aux() {
  return EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_GATE || EPI == MMS_EPI_RELU_DROP_BWD ||
         EPI == MMS_EPI_F16_ACC || EPI == MMS_EPI_GELU_DROP_BWD;
}

// the deferred epilogue operands of one fragment: lane's 4 columns of row m
struct DpAux {
  h16x4 a, b, bias;
};

typedef unsigned int u32x2_dp __attribute__((ext_vector_type(2)));
constexpr int kOut = (int)0x80000000;   // an offset past any extent (the host keeps extents < 2^31 bytes)

// the epilogue's operands as buffer descriptors over their exact extents: a load past the extent
// returns zero and a store past it is dropped, so every wave issues the same loads / stores
// whatever its rows and columns
struct DpRes {
  __amdgpu_buffer_rsrc_t c, o2, aux, bias;
};
MMS_DEV __amdgpu_buffer_rsrc_t dp_rsrc(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, p ? (int)bytes : 0, 0x00020000);
}
MMS_DEV h16x4 dp_ld8(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(h16x4, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
MMS_DEV void dp_st8(__amdgpu_buffer_rsrc_t r, int off, h16x4 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_dp, v), r, off, 0, 0);
}

// fragment (i, j) of a wave's 64x64 accumulator tile: lane owns row (i*16 + (lane & 15)),
// columns j*16 + 4*(lane >> 4) .. +3 (the (B, A)-swapped MFMA layout)
template <int EPI>
MMS_DEV DpAux dp_load(const GemmP& P, const DpRes& R, int m, int n) {
  DpAux x;
  const h16x4 z = {(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
  x.a = z;
  x.b = z;
  x.bias = z;
  const bool ok = m < P.M && n < P.N;
  if (EPI != MMS_EPI_RELU_DROP_BWD && EPI != MMS_EPI_GELU_DROP_BWD) x.bias = dp_ld8(R.bias, ok ? n * 2 : kOut);
  if (!dp_aux<EPI>()) return x;
  if (EPI == MMS_EPI_F16_ACC) {
    x.a = dp_ld8(R.c, ok ? (int)(((long)m * P.ldc + n) * 2) : kOut);
  } else {
    x.a = dp_ld8(R.aux, ok ? (int)(((long)m * P.ldaux + n) * 2) : kOut);
    if (EPI == MMS_EPI_GATE) x.b = dp_ld8(R.aux, ok ? (int)(((long)m * P.ldaux + P.N + n) * 2) : kOut);
  }
  return x;
}

// staged_epilogue's per-element arithmetic (fast path) on 4 consecutive columns; the fp16 results
// and their byte offsets (past the extent for an element outside C: the store is dropped) wait in
// registers for dp_commit at the top of the next k-step.
struct DpOut {
  h16x4 o, o2;
  int off, off2;
};
template <int EPI>
MMS_DEV DpOut dp_compute(const GemmP& P, bool live, int m, int n, const f32x4& v, const DpAux& ax, uint32_t hmix,
                         bool same_hi, bool fast, uint32_t pfrag, float dscale) {
  const bool ok = live && m < P.M && n < P.N;
  DpOut d;
  d.off = ok ? (int)(((long)m * P.ldc + n) * 2) : kOut;
  d.off2 = ok ? (int)(((long)m * P.ldo2 + n) * 2) : kOut;
  float bv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bv[e] = (float)ax.bias[e];
  float x[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] = v[e] * P.alpha + bv[e];
  bool keep[4] = {true, true, true, true};
  if (epi_drops<EPI>() && P.thresh) {
    if (fast) {
      // wave-uniform fast path: the fragment's first pair index comes precomputed (32-bit, no
      // 64-bit counter math); bit-identical to mms_keep4_hi on an even counter
      const uint32_t h0 = mms_mix32(pfrag ^ hmix), h1 = mms_mix32((pfrag + 1) ^ hmix);
      keep[0] = (h0 & 0xffffU) >= P.thresh;
      keep[1] = (h0 >> 16) >= P.thresh;
      keep[2] = (h1 & 0xffffU) >= P.thresh;
      keep[3] = (h1 >> 16) >= P.thresh;
    } else {
      const uint64_t c0 = P.offset + (uint64_t)m * P.ld_rng + n;
      if (same_hi) mms_keep4_hi(hmix, c0, P.thresh, keep);
      else mms_keep4(P.seed, c0, P.thresh, keep);
    }
  }
  h16x4 o4;
  if (EPI == MMS_EPI_GATE) {
    h16x4 g4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float g = sigmoidf_(x[e]), ov = (float)ax.a[e], tv = (float)ax.b[e];
      g4[e] = (h16)g;
      o4[e] = (h16)(tv + g * (ov - tv));
    }
    d.o2 = g4;
  } else if (EPI == MMS_EPI_GELU_DROP) {
    h16x4 z4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      z4[e] = (h16)x[e];
      o4[e] = (h16)(keep[e] ? gelu_((float)z4[e]) * dscale : 0.f);
    }
    d.o2 = z4;
  } else if (EPI == MMS_EPI_GELU_DROP_BWD) {
#pragma unroll
    for (int e = 0; e < 4; ++e) o4[e] = (h16)(keep[e] ? x[e] * dscale * gelu_grad_((float)ax.a[e]) : 0.f);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float o;
      if (EPI == MMS_EPI_RELU_DROP) o = keep[e] ? fmaxf(x[e], 0.f) * dscale : 0.f;
      else if (EPI == MMS_EPI_DROP_RESID) o = (float)ax.a[e] + (keep[e] ? x[e] * dscale : 0.f);
      else if (EPI == MMS_EPI_RELU_DROP_BWD) o = (float)ax.a[e] > 0.f ? x[e] * dscale : 0.f;
      else if (EPI == MMS_EPI_F16_ACC) o = (float)ax.a[e] + x[e];
      else o = x[e];
      o4[e] = (h16)o;
    }
  }
  d.o = o4;
  return d;
}
template <int EPI>
MMS_DEV void dp_commit(const DpRes& R, const DpOut& d) {
  if (EPI == MMS_EPI_GATE || EPI == MMS_EPI_GELU_DROP) dp_st8(R.o2, d.off2, d.o2);
  dp_st8(R.c, d.off, d.o);
}

// XCD-local tile queue: the XCD's contiguous share of the tile space (tile_coords' bijective split)
// is handed out by an atomic ticket counter, one per XCD and launch slot, so a block that starts
// late (its CU held by the side stream's weight gradients) takes fewer tiles instead of delaying
// the launch by a fixed share.  Local ids follow tile_coords' grouped order (GROUP_M tile-rows,
// column by column).  Every block draws exactly one ticket past the end; the block drawing the
// last of those (len + blocks of the XCD - 1) resets the counter for the slot's next launch.
constexpr int DP_SLOTS = 64;
__device__ int g_dp_tickets[DP_SLOTS * 8 * 32];   // one counter per 128-B line

struct DpQueue {
  int* ctr;
  int start, len, gx;
};
MMS_DEV DpQueue dp_queue(int total, int slot) {
  const int x = blockIdx.x % 8, q = total / 8, r = total % 8;
  DpQueue Q;
  Q.ctr = g_dp_tickets + (slot * 8 + x) * 32;
  Q.start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  Q.len = q + (x < r ? 1 : 0);
  Q.gx = gridDim.x / 8 + ((int)(gridDim.x % 8) > x ? 1 : 0);   // blocks on this XCD's queue
  return Q;
}
// The ticket traffic is inline asm, invisible to the compiler's waitcnt pass: as builtins, the
// atomic optimizer turned the one-lane draw into a wave-aggregated atomic whose result it consumed
// at once (vmcnt(0) in front of the k-step's DMA), and the ticket's LDS word made every fragment
// read wait for the in-flight DMA stage.  The draw is issued before a k-step's DMA and retired by
// the next k-step's counted wait (it is older than every operation that wait leaves in flight);
// dp_sync re-defines its result after that wait so no use can be scheduled above it.
MMS_DEV int dp_draw(const DpQueue& Q) {
  int t;
  const int one = 1;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(t) : "v"(Q.ctr), "v"(one) : "memory");
  return t;
}
MMS_DEV void dp_sync(int& t) { asm volatile("" : "+v"(t)); }
MMS_DEV void dp_retire(const DpQueue& Q, int t) {   // after every draw, once its value is back
  if (t == Q.len + Q.gx - 1) {
    const int zero = 0;
    asm volatile("global_atomic_swap %0, %1, off" :: "v"(Q.ctr), "v"(zero) : "memory");
  }
}
MMS_DEV void dp_put(char* lds, int t) {
  asm volatile("ds_write_b32 %0, %1" :: "v"((unsigned)(uintptr_t)lds), "v"(t) : "memory");
}
MMS_DEV int dp_get(const char* lds) {
  int t;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"((unsigned)(uintptr_t)lds) : "memory");
  return t;
}
MMS_DEV bool dp_tile(const DpQueue& Q, int ticket, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  if (ticket >= Q.len) return false;
  const int t = Q.start + ticket;
  const int per_group = group_m * tiles_n;
  const int g = t / per_group, first_m = g * group_m;
  const int gsize = min(tiles_m - first_m, group_m);
  const int w = t % per_group;
  tm = first_m + w % gsize;
  tn = w / gsize;
  return true;
}

// k-steps 0 .. NP-1 with compile-time step numbers (they carry the deferred fragments), straight-
// line: the host routes only K >= (NP_ + 2) * 64 here, so every one of them runs and DMAs the same
// tile's next stage (a conditional step would merge wait states and cost vmcnt waits on the DMA)
template <int U, int NP, typename F>
MMS_DEV void unroll_ksteps(F& f) {
  if constexpr (U < NP) {
    f(U, std::integral_constant<int, U>{});
    unroll_ksteps<U + 1, NP>(f);
  }
}

template <int EPI>
__global__ void __launch_bounds__(NT, 2) gemm_dp_kernel(GemmP P, int tiles_m, int tiles_n, int total, int slot) {
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES + 16];   // + the next tile's ticket
  char* const s_ticket = smem + 2 * 2 * TILE_BYTES;
#define SA(s) (smem + (2 * (s)) * TILE_BYTES)
#define SB(s) (smem + (2 * (s) + 1) * TILE_BYTES)
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.A, (short)0, (int)(((long)(P.M - 1) * P.lda + P.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P.B, (short)0, (int)(((long)(P.N - 1) * P.ldb + P.K) * 2), 0x00020000);
  DpRes R;
  R.c = dp_rsrc(P.C, ((long)(P.M - 1) * P.ldc + P.N) * 2);
  R.o2 = dp_rsrc(P.out2, ((long)(P.M - 1) * P.ldo2 + P.N) * 2);
  R.aux = dp_rsrc(P.aux, ((long)(P.M - 1) * P.ldaux + (EPI == MMS_EPI_GATE ? 2 : 1) * P.N) * 2);
  R.bias = dp_rsrc(P.bias, (long)P.N * 2);
  const int nk = P.K / BK;   // host: K % 64 == 0, nk >= NP_ + 2
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;

  const DpQueue Q = dp_queue(total, slot);
  if (threadIdx.x == 0) {
    int t = dp_draw(Q);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dp_sync(t);
    dp_retire(Q, t);
    dp_put(s_ticket, t);
  }
  __syncthreads();
  int tm, tn;
  if (!dp_tile(Q, dp_get(s_ticket), tiles_m, tiles_n, P.group_m, tm, tn)) {
    stamp_end(P.stamps, t_start);
    return;
  }
  // the next tile's ticket: drawn by thread 0 in a tile's k-step 0, parked in LDS in k-step 1
  // (behind that step's vmcnt(0)), read by every thread in the last k-step
  int ticket_req = 0;
  dma_tile<true>(ra, SA(0), P.lda, tm * BM, 0, wid, lane);
  dma_tile<true>(rb, SB(0), P.ldb, tn * BN, 0, wid, lane);

  // the previous tile's accumulators and its epilogue state
  f32x4 prev[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) prev[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int pm0 = 0, pn0 = 0;   // lane's first row / column of the previous tile
  bool have_prev = false;
  uint32_t hmix = 0, pbase = 0;   // pbase: the lane's first dropout pair index (fast path)
  bool same_hi = false, fast = false;
  // operands of the fragments finished in k-step e live in pa[e & 1]: the next k-step's are loaded
  // while this one's are consumed
  DpAux pa[2][DP_PIECES];
  {
    const h16x4 z = {(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int u = 0; u < DP_PIECES; ++u) pa[b][u] = DpAux{z, z, z};
  }
  // fragment p = 4 i + j of the previous tile (p compile-time after unrolling)
  auto load_pieces = [&](int p0) __attribute__((always_inline)) {
    DpAux* dst = pa[(p0 / DP_PIECES) & 1];
#pragma unroll
    for (int u = 0; u < DP_PIECES; ++u)
      if (p0 + u < 16) dst[u] = dp_load<EPI>(P, R, pm0 + ((p0 + u) >> 2) * 16, pn0 + ((p0 + u) & 3) * 16);
  };
  // the previous tile's fragments p0 .. p0 + DP_PIECES - 1 (also on the first tile, dropped there)
  DpOut po[DP_PIECES];
  auto compute_pieces = [&](int p0) __attribute__((always_inline)) {
    const DpAux* src = pa[(p0 / DP_PIECES) & 1];
#pragma unroll
    for (int u = 0; u < DP_PIECES; ++u) {
      const int p = p0 + u;
      if (p < 16) {
        const uint32_t pfrag = pbase + (uint32_t)((p >> 2) * 8) * (uint32_t)P.ld_rng + (uint32_t)((p & 3) * 8);
        po[u] = dp_compute<EPI>(P, have_prev, pm0 + (p >> 2) * 16, pn0 + (p & 3) * 16, prev[p >> 2][p & 3], src[u],
                                hmix, same_hi, fast, pfrag, dscale);
      }
    }
  };
  auto commit_pieces = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < DP_PIECES; ++u) dp_commit<EPI>(R, po[u]);
  };

  int kbase = 0;   // k-steps run so far: the ring parity carries over from tile to tile
  for (;;) {
    const int bm = tm * BM, bn = tn * BN;
    int ntm = 0, ntn = 0;
    bool more = false;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    load_pieces(0);
    // one k-step; EP >= 0: also finish the previous tile's fragments EP*DP_PIECES.. (EP compile-time):
    // their arithmetic runs after the k-step's MFMAs are issued (beside the matrix core), their
    // stores at the top of the next k-step together with the DMA, so both have a whole k-step to
    // land before its vmcnt(0) (the wait makes no assumption about the order in which loads,
    // stores and atomics retire).  Aux operands are loaded one k-step ahead of their arithmetic.
    auto kstep = [&](int kt, auto ep) __attribute__((always_inline)) {
      constexpr int EP = decltype(ep)::value;
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int cur = (kbase + kt) & 1;
      if (EP >= 1 && EP <= NP_) commit_pieces();
      if (EP == 0 && threadIdx.x == 0) ticket_req = dp_draw(Q);
      if (EP == 1 && threadIdx.x == 0) {
        dp_sync(ticket_req);
        dp_retire(Q, ticket_req);
        dp_put(s_ticket, ticket_req);
      }
      if (EP < 0 && kt == nk - 1) more = dp_tile(Q, dp_get(s_ticket), tiles_m, tiles_n, P.group_m, ntm, ntn);
      if (EP >= 0 || kt + 1 < nk) {
        dma_tile<true>(ra, SA(cur ^ 1), P.lda, bm, (kt + 1) * BK, wid, lane);
        dma_tile<true>(rb, SB(cur ^ 1), P.ldb, bn, (kt + 1) * BK, wid, lane);
      } else if (more) {   // the next tile's first stage, behind this tile's last k-step
        dma_tile<true>(ra, SA(cur ^ 1), P.lda, ntm * BM, 0, wid, lane);
        dma_tile<true>(rb, SB(cur ^ 1), P.ldb, ntn * BN, 0, wid, lane);
      }
      // (issued on the first tile as well, over row / column 0: the loads stay unconditional)
      if (EP >= 0 && EP < NP_ && (EP + 1) * DP_PIECES < 16) load_pieces((EP + 1) * DP_PIECES);
      // keep the stores / DMA / aux loads at the top: the scheduler would otherwise sink the stores
      // behind the MFMAs and shorten the time they have before the next k-step's vmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
      h16x8 fa2[2][4], fb2[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa2[kk][i] = read_frag<true>(SA(cur), wm * 64 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb2[kk][j] = read_frag<true>(SB(cur), wn * 64 + j * 16, kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb2[kk][j], fa2[kk][i], acc[i][j], 0, 0, 0);
      if (EP >= 0 && EP < NP_) compute_pieces(EP * DP_PIECES);
    };
    // k-steps 0 .. NP_-1 carry deferred fragments; step NP_ (no fragments) still waits behind the
    // previous step's stores; the rest wait for everything (EP = -1)
    unroll_ksteps<0, NP_ + 1>(kstep);
    for (int kt = NP_ + 1; kt < nk; ++kt) kstep(kt, std::integral_constant<int, -1>{});
    kbase += nk;
    // this tile becomes the deferred one
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) prev[i][j] = acc[i][j];
    pm0 = bm + wm * 64 + (lane & 15);
    pn0 = bn + wn * 64 + 4 * (lane >> 4);
    have_prev = true;
    if (epi_drops<EPI>() && P.thresh) {
      // one hash half per lane and tile when every counter of the lane's fragments shares the
      // high word (staged_epilogue's fast path; bit-identical to mms_keep4)
      const uint64_t cf = P.offset + (uint64_t)pm0 * P.ld_rng + pn0;
      const uint64_t cl = P.offset + (uint64_t)(pm0 + 48) * P.ld_rng + pn0 + 48 + 3;
      same_hi = mms_same_hi(cf, cl) && ((cf & 1) == 0) && ((P.ld_rng & 1) == 0);
      hmix = mms_hi_mix(P.seed, cf);
      pbase = (uint32_t)(cf >> 1);
      fast = __all(same_hi);
    }
    if (!more) break;
    tm = ntm;
    tn = ntn;
  }
  // the last tile's epilogue
  __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
  for (int p0 = 0; p0 < 16; p0 += DP_PIECES) {
    load_pieces(p0);
    compute_pieces(p0);
    commit_pieces();
  }
#undef SA
#undef SB
  stamp_end(P.stamps, t_start);
}

}  // namespace

namespace mmsg {
int launch_dp(int epi, const GemmP& P, int tiles_m, int tiles_n, int grid, hipStream_t s) {
  const int total = tiles_m * tiles_n;
  // ticket-counter slot: launches in flight at once (main and side stream) never share one
  static std::atomic<unsigned> next_slot{0};
  const int slot = (int)(next_slot.fetch_add(1, std::memory_order_relaxed) % DP_SLOTS);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_dp_kernel<E>), dim3(grid), dim3(NT), 0, s, P, tiles_m, tiles_n, total, slot); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_GATE)
    CASE(MMS_EPI_RELU_DROP_BWD) CASE(MMS_EPI_F16_ACC) CASE(MMS_EPI_GELU_DROP) CASE(MMS_EPI_GELU_DROP_BWD)
#undef CASE
    default: mms::set_error("gemm_dp: bad epilogue %d", epi); return 1;
  }
  return mms::check_launch("gemm_dp");
}
}  // namespace mmsg
