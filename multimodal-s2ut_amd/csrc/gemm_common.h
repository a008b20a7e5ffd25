// Shared pieces of the MFMA GEMM kernels (gemm.hip: 128x128 / tall / 256x256 tiles; the GEMM lab,
// scripts/micro): launch parameters, tile order, LDS fragment reads, fused epilogues.  Everything
// but GemmP has internal linkage.
#pragma once
#include "common.h"
#include "../../include/mms2ut.h"

// Launch parameters of every GEMM kernel
namespace mmsg {
struct GemmP {
  const h16* A; const h16* B; void* C;
  int M, N, K;
  long lda, ldb, ldc;
  int bdiv;  // batch index z -> (z / bdiv, z % bdiv)
  long sA1, sA2, sB1, sB2, sC1, sC2;
  int splitk; int kchunk; long sCsplit;
  // epilogue
  float alpha;
  const h16* bias;
  const h16* aux; long ldaux; long sX1, sX2;
  h16* out2; long ldo2;
  float p; uint32_t thresh; uint64_t seed, offset; long ld_rng;
  int vec16;  // every fp16 row operand of the epilogue is 16-B aligned at 8-column granularity (3: and
              // the fp32-staged epilogue forced, mms2ut_gemm_set_epilogue)
  float* rowsum; long ld_rowsum;  // RS kernels: split-K partial A-row sums (bias gradient)
  h16* rowsum16;                  // RS kernels, unsplit: the fp16 A-row sums (grouped wgrad)
  int group_m;  // tile-rows per L2 group (tile_coords)
  unsigned long long* stamps;  // profiling: per block {first, last} s_memrealtime tick, or null
};

}  // namespace mmsg

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
#ifndef MMS_GEMM_PRIO
#define MMS_GEMM_PRIO 1
#endif
// raise wave priority around the MFMA block of a k-step — for the fp16-output (forward / dgrad,
// critical-path) GEMMs only, so that their waves win issue slots over the side stream's
// weight-gradient (fp32 slab) GEMM waves sharing a CU
constexpr bool PRIO = MMS_GEMM_PRIO;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KiB per operand per stage

using mmsg::GemmP;

// Live kernel timing (bench roofline): with P.stamps set, thread 0 of every block stores the
// block's start tick and its end tick (after the block's last global store has completed) at
// stamps[2 * blockIdx.x].  A launch's duration is max(end) - min(start) over its blocks — the
// dispatch span rocprofv3's kernel trace reports, measured inside the real (overlapped) step.
// One 16-B store per block; nothing is recorded when stamps is null.
MMS_DEV unsigned long long stamp_now() { return __builtin_amdgcn_s_memrealtime(); }
MMS_DEV void stamp_end(unsigned long long* stamps, unsigned long long t0) {
  if (!stamps) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t1 = stamp_now();
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    *reinterpret_cast<u64x2*>(stamps + 2 * (long)blockIdx.x) = u64x2{t0, t1};
  }
}

MMS_DEV int swz_mn(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

// fragment for rows [sub, sub+16) and k in [kk*32, kk*32+32): lane l holds X(sub + (l&15), kk*32 + 8(l>>4) + j)
template <bool KC>
MMS_DEV h16x8 read_frag(const char* lds, int sub, int kk, int lane) {
  if (KC) {
    const int r = sub + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    s16x8 v = *reinterpret_cast<const s16x8*>(lds + r * 128 + ((c ^ (r & 7)) << 4));
    return __builtin_bit_cast(h16x8, v);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int col = sub + 4 * p;                // element column (row of the logical operand)
    const int chunk = col >> 3, inb = (col & 7) * 2;
    const int k1 = kk * 32 + 8 * g + q, k2 = k1 + 4;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const char* a1 = lds + k1 * 256 + ((chunk ^ swz_mn(k1)) << 4) + inb;
    const char* a2 = lds + k2 * 256 + ((chunk ^ swz_mn(k2)) << 4) + inb;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a2));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(h16x8, v);
  }
}

MMS_DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
// torch F.gelu (approximate='none'): 0.5 z (1 + erf(z / sqrt 2)) and its derivative
MMS_DEV float gelu_(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }
MMS_DEV float gelu_grad_(float z) {
  return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.39894228040143268f * __expf(-0.5f * z * z);
}

template <int EPI>
MMS_DEV void epilogue_store(const GemmP& P, void* Cz, const h16* auxz, int m, int n, f32x4 v) {
  if (m >= P.M) return;
  const int N = P.N;
  float x[4] = {v[0] * P.alpha, v[1] * P.alpha, v[2] * P.alpha, v[3] * P.alpha};
  if (EPI == MMS_EPI_F32) {
    float* C = reinterpret_cast<float*>(Cz) + (long)m * P.ldc;
    if (n + 3 < N) {
      *reinterpret_cast<f32x4*>(C + n) = f32x4{x[0], x[1], x[2], x[3]};
    } else {
      for (int r = 0; r < 4; ++r) if (n + r < N) C[n + r] = x[r];
    }
    return;
  }
  const bool full = n + 3 < N;
  if (P.bias && EPI != MMS_EPI_RELU_DROP_BWD && EPI != MMS_EPI_GELU_DROP_BWD) {
    if (full) {
      const h16x4 bv = *reinterpret_cast<const h16x4*>(P.bias + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] += (float)bv[r];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) if (n + r < N) x[r] += (float)P.bias[n + r];
    }
  }
  h16* C = reinterpret_cast<h16*>(Cz) + (long)m * P.ldc;
  // 4-wide operand fetches (aux row / existing C), zero beyond N
  auto ld4 = [&](const h16* row, int col, float (&v)[4]) {
    if (full) {
      const h16x4 t = *reinterpret_cast<const h16x4*>(row + col);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (float)t[r];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (n + r < N) ? (float)row[col + r] : 0.f;
    }
  };
  bool keep[4] = {true, true, true, true};
  if ((EPI == MMS_EPI_RELU_DROP || EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_GELU_DROP ||
       EPI == MMS_EPI_GELU_DROP_BWD) && P.thresh)
    mms_keep4(P.seed, P.offset + (uint64_t)m * P.ld_rng + n, P.thresh, keep);
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  float o[4];
  if (EPI == MMS_EPI_RELU_DROP) {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = keep[r] ? fmaxf(x[r], 0.f) * dscale : 0.f;
  } else if (EPI == MMS_EPI_DROP_RESID) {
    float a[4];
    ld4(auxz + (long)m * P.ldaux, n, a);
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = a[r] + (keep[r] ? x[r] * dscale : 0.f);
  } else if (EPI == MMS_EPI_GATE) {
    float ov[4], tv[4];
    ld4(auxz + (long)m * P.ldaux, n, ov);
    ld4(auxz + (long)m * P.ldaux + N, n, tv);
    float g[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      g[r] = sigmoidf_(x[r]);
      o[r] = tv[r] + g[r] * (ov[r] - tv[r]);
    }
    h16* g_row = P.out2 + (long)m * P.ldo2;
    if (full) {
      *reinterpret_cast<h16x4*>(g_row + n) = h16x4{(h16)g[0], (h16)g[1], (h16)g[2], (h16)g[3]};
    } else {
      for (int r = 0; r < 4; ++r) if (n + r < N) g_row[n + r] = (h16)g[r];
    }
  } else if (EPI == MMS_EPI_RELU_DROP_BWD) {
    float h[4];
    ld4(auxz + (long)m * P.ldaux, n, h);
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = h[r] > 0.f ? x[r] * dscale : 0.f;
  } else if (EPI == MMS_EPI_F16_ACC) {
    float c[4];
    ld4(C, n, c);
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = c[r] + x[r];
  } else if (EPI == MMS_EPI_GELU_DROP) {
    h16 zh[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      zh[r] = (h16)x[r];
      o[r] = keep[r] ? gelu_((float)zh[r]) * dscale : 0.f;
    }
    h16* z_row = P.out2 + (long)m * P.ldo2;
    if (full) {
      *reinterpret_cast<h16x4*>(z_row + n) = h16x4{zh[0], zh[1], zh[2], zh[3]};
    } else {
      for (int r = 0; r < 4; ++r) if (n + r < N) z_row[n + r] = zh[r];
    }
  } else if (EPI == MMS_EPI_GELU_DROP_BWD) {
    float z[4];
    ld4(auxz + (long)m * P.ldaux, n, z);
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = keep[r] ? x[r] * dscale * gelu_grad_(z[r]) : 0.f;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = x[r];
  }
  if (full) {
    *reinterpret_cast<h16x4*>(C + n) = h16x4{(h16)o[0], (h16)o[1], (h16)o[2], (h16)o[3]};
  } else {
    for (int r = 0; r < 4; ++r) if (n + r < N) C[n + r] = (h16)o[r];
  }
}

// 8 consecutive columns n..n+7 (n % 8 == 0) of row m: 16-B operand loads / stores when aligned,
// otherwise two 4-wide calls of epilogue_store (which also handles the N tail)
template <int EPI>
MMS_DEV void epilogue_store8(const GemmP& P, void* Cz, const h16* auxz, int m, int n, const float (&v)[8]) {
  if (m >= P.M || n >= P.N) return;
  const int N = P.N;
  if (EPI == MMS_EPI_F32) {
    float* C = reinterpret_cast<float*>(Cz) + (long)m * P.ldc;
    if (n + 7 < N) {
      *reinterpret_cast<f32x4*>(C + n) = f32x4{v[0] * P.alpha, v[1] * P.alpha, v[2] * P.alpha, v[3] * P.alpha};
      *reinterpret_cast<f32x4*>(C + n + 4) = f32x4{v[4] * P.alpha, v[5] * P.alpha, v[6] * P.alpha, v[7] * P.alpha};
    } else {
      for (int r = 0; r < 8; ++r) if (n + r < N) C[n + r] = v[r] * P.alpha;
    }
    return;
  }
  if (!(P.vec16 && n + 7 < N)) {
    epilogue_store<EPI>(P, Cz, auxz, m, n, f32x4{v[0], v[1], v[2], v[3]});
    epilogue_store<EPI>(P, Cz, auxz, m, n + 4, f32x4{v[4], v[5], v[6], v[7]});
    return;
  }
  float x[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) x[r] = v[r] * P.alpha;
  if (P.bias && EPI != MMS_EPI_RELU_DROP_BWD && EPI != MMS_EPI_GELU_DROP_BWD) {
    const h16x8 bv = *reinterpret_cast<const h16x8*>(P.bias + n);
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] += (float)bv[r];
  }
  h16* C = reinterpret_cast<h16*>(Cz) + (long)m * P.ldc;
  auto ld8 = [&](const h16* src, float (&o)[8]) {
    const h16x8 t = *reinterpret_cast<const h16x8*>(src);
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = (float)t[r];
  };
  bool keep[8] = {true, true, true, true, true, true, true, true};
  if ((EPI == MMS_EPI_RELU_DROP || EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_GELU_DROP ||
       EPI == MMS_EPI_GELU_DROP_BWD) && P.thresh) {
    const uint64_t c0 = P.offset + (uint64_t)m * P.ld_rng + n;
    bool k0[4], k1[4];
    mms_keep4(P.seed, c0, P.thresh, k0);
    mms_keep4(P.seed, c0 + 4, P.thresh, k1);
#pragma unroll
    for (int r = 0; r < 4; ++r) { keep[r] = k0[r]; keep[r + 4] = k1[r]; }
  }
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  float o[8];
  if (EPI == MMS_EPI_RELU_DROP) {
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = keep[r] ? fmaxf(x[r], 0.f) * dscale : 0.f;
  } else if (EPI == MMS_EPI_DROP_RESID) {
    float a[8];
    ld8(auxz + (long)m * P.ldaux + n, a);
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = a[r] + (keep[r] ? x[r] * dscale : 0.f);
  } else if (EPI == MMS_EPI_GATE) {
    float ov[8], tv[8], g[8];
    ld8(auxz + (long)m * P.ldaux + n, ov);
    ld8(auxz + (long)m * P.ldaux + N + n, tv);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      g[r] = sigmoidf_(x[r]);
      o[r] = tv[r] + g[r] * (ov[r] - tv[r]);
    }
    h16x8 gv;
#pragma unroll
    for (int r = 0; r < 8; ++r) gv[r] = (h16)g[r];
    *reinterpret_cast<h16x8*>(P.out2 + (long)m * P.ldo2 + n) = gv;
  } else if (EPI == MMS_EPI_RELU_DROP_BWD) {
    float h[8];
    ld8(auxz + (long)m * P.ldaux + n, h);
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = h[r] > 0.f ? x[r] * dscale : 0.f;
  } else if (EPI == MMS_EPI_F16_ACC) {
    float c[8];
    ld8(C + n, c);
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = c[r] + x[r];
  } else if (EPI == MMS_EPI_GELU_DROP) {
    h16x8 zv;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      zv[r] = (h16)x[r];
      o[r] = keep[r] ? gelu_((float)zv[r]) * dscale : 0.f;
    }
    *reinterpret_cast<h16x8*>(P.out2 + (long)m * P.ldo2 + n) = zv;
  } else if (EPI == MMS_EPI_GELU_DROP_BWD) {
    float z[8];
    ld8(auxz + (long)m * P.ldaux + n, z);
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = keep[r] ? x[r] * dscale * gelu_grad_(z[r]) : 0.f;
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = x[r];
  }
  h16x8 ov8;
#pragma unroll
  for (int r = 0; r < 8; ++r) ov8[r] = (h16)o[r];
  *reinterpret_cast<h16x8*>(C + n) = ov8;
}

// Epilogue through LDS: each wave parks its 64x64 fp32 accumulator tile in 16 KiB of the (now idle)
// operand ring, XOR-swizzled by row, then re-reads it row-major so a lane owns 8 consecutive
// columns: every global load/store of the epilogue covers whole 128-B row segments instead of
// 16 rows x 32 B.  Caller guarantees all waves are past their last operand read.
// Block -> (z, tm, tn).  The grid is 1-D over tiles_m * tiles_n * nz.  Workgroups are dispatched
// round-robin over the 8 XCDs, each with a private 4 MiB L2, so the linear id is first remapped
// (bijectively) to give every XCD one contiguous range of the z-major tile space: a split-K
// slice, or a batch entry, stays on one XCD.  Inside a z slice tiles go in groups of GROUP_M
// tile-rows, column by column, so the ~64 blocks an XCD runs at once share 8 A row-panels and 8
// B column-panels (~3 MiB at K = 768) instead of streaming the whole B operand per row.
MMS_DEV void tile_coords(int bid, int tiles_m, int tiles_n, int total, int& z, int& tm, int& tn, int GROUP_M) {
  const int q = total / 8, r = total % 8, x = bid % 8;
  const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  const int ntiles = tiles_m * tiles_n;
  z = id / ntiles;
  const int t = id % ntiles;
  const int per_group = GROUP_M * tiles_n;
  const int g = t / per_group, first_m = g * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int w = t % per_group;
  tm = first_m + w % gsize;
  tn = w / gsize;
}

template <int EPI>
constexpr bool epi_drops() {
  return EPI == MMS_EPI_RELU_DROP || EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_GELU_DROP ||
         EPI == MMS_EPI_GELU_DROP_BWD;
}

// Register epilogue (round 6): for the epilogues whose element math needs no operand in row-major
// order (plain / bias, ReLU-dropout) the math runs on the accumulators in the MFMA layout (lane l:
// row 16 i + (l & 15), columns 16 j + 4 (l >> 4) .. + 3), the fp16 results go through the wave's own
// LDS slot (FR x 16 rows x 128 B, half the bytes of the fp32 staging, one pass for up to 8 fragments)
// and come back row-major for 16-B stores of whole 128-B row segments.  Same per-element arithmetic
// and the same dropout counters as the staged path: bit-identical.  The slot is written and read by
// one wave only, so no workgroup barrier sits between the two.
#ifndef MMS_GEMM_REG_EPI
#define MMS_GEMM_REG_EPI 1
#endif
#ifndef MMS_GEMM_REG_STAGED
#define MMS_GEMM_REG_STAGED 1
#endif
#ifndef MMS_GEMM_REG_TALL
#define MMS_GEMM_REG_TALL 1
#endif
template <int EPI>
constexpr bool epi_regs() {
  return MMS_GEMM_REG_EPI && (EPI == MMS_EPI_F16 || EPI == MMS_EPI_RELU_DROP);
}

// The choice between this and the staged path must be the same for every wave of a block: the two
// lay their LDS slots out differently (the tall kernel packs the fp16 slots) and the staged path
// holds workgroup barriers.  N % 64 == 0 makes every wave's 64 columns lie wholly inside N or wholly
// outside it (such a wave has nothing to do).
MMS_DEV bool reg_epilogue_ok(const GemmP& P) { return P.vec16 == 1 && P.N % 64 == 0; }   // 3: staged (test hook)

// rows bm + 64 wm + 16 i + (l & 15), columns bn + 64 wn ..+ 64 (caller: reg_epilogue_ok(P));
// SLOTB: bytes between consecutive waves' slots (>= FR * 2048)
template <int EPI, int FR, int SLOTB>
MMS_DEV void reg_epilogue(const GemmP& P, char* smem, const f32x4 (&acc)[FR][4], int bm, int bn, int wm, int wn,
                          int wid, int lane, void* Cz) {
  static_assert(SLOTB >= FR * 2048, "staging slot too small");
  if (bn + wn * 64 >= P.N) return;   // wave-uniform: all 64 columns past N
  char* stage = smem + wid * SLOTB;
  const int rl = lane & 15, g = lane >> 4;
  const int m0 = bm + wm * 64 + rl, nw = bn + wn * 64 + 4 * g;
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = 0.f;
  if (P.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const h16x4 b4 = *reinterpret_cast<const h16x4*>(P.bias + nw + 16 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[j][e] = (float)b4[e];
    }
  }
  constexpr bool DROPS = EPI == MMS_EPI_RELU_DROP;
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  uint32_t hmix = 0, pbase = 0;
  bool fast = false;
  if (DROPS && P.thresh) {
    const uint64_t cf = P.offset + (uint64_t)m0 * P.ld_rng + nw;
    const uint64_t cl = P.offset + (uint64_t)(m0 + 16 * (FR - 1)) * P.ld_rng + nw + 51;
    const bool sh = mms_same_hi(cf, cl) && ((cf & 1) == 0) && ((P.ld_rng & 1) == 0);
    hmix = mms_hi_mix(P.seed, cf);
    pbase = (uint32_t)(cf >> 1);
    fast = __all(sh);
  }
#pragma unroll
  for (int i = 0; i < FR; ++i) {
    const int rr = i * 16 + rl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = acc[i][j][e] * P.alpha + bv[j][e];
      bool keep[4] = {true, true, true, true};
      if (DROPS && P.thresh && fast) {
        // pair index of counter offset + (m0 + 16 i) ld_rng + nw + 16 j (ld_rng even)
        const uint32_t p0 = pbase + (uint32_t)(8 * i) * (uint32_t)P.ld_rng + 8 * j;
        const uint32_t h0 = mms_mix32(p0 ^ hmix), h1 = mms_mix32((p0 + 1) ^ hmix);
        keep[0] = (h0 & 0xffffU) >= P.thresh;
        keep[1] = (h0 >> 16) >= P.thresh;
        keep[2] = (h1 & 0xffffU) >= P.thresh;
        keep[3] = (h1 >> 16) >= P.thresh;
      } else if (DROPS && P.thresh) {
        mms_keep4(P.seed, P.offset + (uint64_t)(m0 + 16 * i) * P.ld_rng + nw + 16 * j, P.thresh, keep);
      }
      h16x4 o4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float o;
        if (EPI == MMS_EPI_RELU_DROP) o = keep[e] ? fmaxf(x[e], 0.f) * dscale : 0.f;
        else o = x[e];
        o4[e] = (h16)o;
      }
      // 16-B chunk 2 j + (g >> 1) of row rr, 8-B half g & 1; chunks XOR-swizzled by (rr >> 1) & 7 and
      // halves by rr & 1: a ds_write_b64 16-lane group (16 rows, one (j, g)) covers the 32 write banks
      // once, ds_read_b128's lane groups read distinct chunks (PMC: SQ_LDS_BANK_CONFLICT 0)
      const int ch = (2 * j + (g >> 1)) ^ ((rr >> 1) & 7);
      *reinterpret_cast<h16x4*>(stage + rr * 128 + (ch << 4) + (((g ^ rr) & 1) << 3)) = o4;
    }
  }
  // the slot is re-read by other lanes of this wave: drain its LDS writes first (DS operations of a
  // wave complete in order, the wait makes that explicit at the cost of one short stall)
  // (same-box A/B with / without the wait: step 15.58-15.60 vs 15.57-15.66 ms, profiles/round6_reg_epilogue_drain_ab.txt)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int q = lane & 7;
  h16* C = reinterpret_cast<h16*>(Cz);
  const int n = bn + wn * 64 + 8 * q;
#pragma unroll
  for (int pass = 0; pass < 2 * FR; ++pass) {
    const int rr = pass * 8 + (lane >> 3);
    typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
    u32x4_ v = *reinterpret_cast<const u32x4_*>(stage + rr * 128 + ((q ^ ((rr >> 1) & 7)) << 4));
    if (rr & 1) v = u32x4_{v[2], v[3], v[0], v[1]};   // odd rows store their two halves swapped
    const int m = bm + wm * 64 + rr;
    if (m < P.M) *reinterpret_cast<u32x4_*>(C + (long)m * P.ldc + n) = v;
  }
}

// FR: 16-row fragments of the wave's tile in this pass (4 = 64 rows; 2 = 32 rows); SLOT: floats of
// LDS between consecutive waves' staging areas (>= FR * 16 * 64)
template <int EPI, int FR = 4, int SLOT = 64 * 64>
MMS_DEV void staged_epilogue(const GemmP& P, char* smem, const f32x4 (&acc)[FR][4], int bm, int bn,
                             int wm, int wn, int wid, int lane, void* Cz, const h16* auxz) {
  static_assert(SLOT >= FR * 16 * 64, "staging slot too small");
  if constexpr (epi_regs<EPI>() && MMS_GEMM_REG_STAGED) {
    if (reg_epilogue_ok(P)) {   // launch-uniform: every wave of the block takes the same path
      reg_epilogue<EPI, FR, SLOT * 4>(P, smem, acc, bm, bn, wm, wn, wid, lane, Cz);
      return;
    }
  }
  constexpr int PASSES = FR * 2;   // 8 rows per pass
  float* stage = reinterpret_cast<float*>(smem) + wid * SLOT;
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = i * 16 + (lane & 15);
      const int c = j * 4 + (lane >> 4);
      *reinterpret_cast<f32x4*>(stage + r * 64 + ((c ^ (r & 15)) << 2)) = acc[i][j];
    }
  __syncthreads();
  const int q = lane & 7;
  const int n = bn + wn * 64 + 8 * q;
  auto stage8 = [&](int r, float (&v)[8]) {
    const f32x4 lo = *reinterpret_cast<const f32x4*>(stage + r * 64 + (((2 * q) ^ (r & 15)) << 2));
    const f32x4 hi = *reinterpret_cast<const f32x4*>(stage + r * 64 + (((2 * q + 1) ^ (r & 15)) << 2));
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  };
  constexpr bool LOADS = EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_GATE || EPI == MMS_EPI_RELU_DROP_BWD ||
                         EPI == MMS_EPI_F16_ACC || EPI == MMS_EPI_GELU_DROP_BWD;
  if (EPI == MMS_EPI_F32 || !(P.vec16 && n + 7 < P.N)) {
#pragma unroll 2
    for (int pass = 0; pass < PASSES; ++pass) {
      const int r = pass * 8 + (lane >> 3);
      float v[8];
      stage8(r, v);
      epilogue_store8<EPI>(P, Cz, auxz, bm + wm * 64 + r, n, v);
    }
    return;
  }
  // Fast path (every fp16 row operand 16-B aligned, 8 whole columns): the global operand loads of
  // all 8 rows (aux / existing C, bias) are issued before the first store.  Interleaved per row,
  // hipcc must keep each row's loads behind the previous row's stores (they may alias), which
  // serialised the epilogue into 8 dependent global round trips.
  const int m0 = bm + wm * 64 + (lane >> 3);
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (EPI != MMS_EPI_RELU_DROP_BWD && EPI != MMS_EPI_GELU_DROP_BWD && P.bias) {
    const h16x8 b8 = *reinterpret_cast<const h16x8*>(P.bias + n);
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = (float)b8[e];
  }
  h16* C = reinterpret_cast<h16*>(Cz);
  h16x8 ax[8], ax2[8];
  const h16x8 z8 = {(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    const int m = m0 + 8 * pass;
    ax[pass] = z8;
    ax2[pass] = z8;
    if (LOADS && m < P.M) {
      if (EPI == MMS_EPI_F16_ACC) {
        ax[pass] = *reinterpret_cast<const h16x8*>(C + (long)m * P.ldc + n);
      } else {
        ax[pass] = *reinterpret_cast<const h16x8*>(auxz + (long)m * P.ldaux + n);
        if (EPI == MMS_EPI_GATE) ax2[pass] = *reinterpret_cast<const h16x8*>(auxz + (long)m * P.ldaux + P.N + n);
      }
    }
  }
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  constexpr bool DROPS = EPI == MMS_EPI_RELU_DROP || EPI == MMS_EPI_DROP_RESID || EPI == MMS_EPI_GELU_DROP ||
                         EPI == MMS_EPI_GELU_DROP_BWD;
  // the seed / high-counter half of the dropout hash is one constant for all 64 of this lane's
  // counters whenever they share the high word (always, unless the run straddles a 2^33
  // boundary): one mixer per pair of elements instead of two (bit-identical to mms_keep4)
  uint32_t hmix = 0, pbase = 0;
  bool same_hi = false, fast = false;
  if (DROPS && P.thresh) {
    const uint64_t cf = P.offset + (uint64_t)m0 * P.ld_rng + n;
    const uint64_t cl = P.offset + (uint64_t)(m0 + 8 * (PASSES - 1)) * P.ld_rng + n + 7;
    same_hi = mms_same_hi(cf, cl) && ((cf & 1) == 0) && ((P.ld_rng & 1) == 0);
    hmix = mms_hi_mix(P.seed, cf);
    // wave-uniform fast path (the compiler versions the pass loop on it): pass p's first pair index
    // is pbase + 4 p ld_rng, in 32-bit arithmetic, no 64-bit counter per pass
    pbase = (uint32_t)(cf >> 1);
    fast = __all(same_hi);
  }
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    const int m = m0 + 8 * pass;
    if (m >= P.M) continue;
    float x[8];
    stage8(pass * 8 + (lane >> 3), x);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = x[e] * P.alpha + bv[e];
    bool keep[8] = {true, true, true, true, true, true, true, true};
    if (DROPS && P.thresh && fast) {
      const uint32_t p0 = pbase + (uint32_t)(4 * pass) * (uint32_t)P.ld_rng;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t hv = mms_mix32((p0 + h) ^ hmix);
        keep[2 * h] = (hv & 0xffffU) >= P.thresh;
        keep[2 * h + 1] = (hv >> 16) >= P.thresh;
      }
    } else if (DROPS && P.thresh) {
      const uint64_t c0 = P.offset + (uint64_t)m * P.ld_rng + n;
      bool k0[4], k1[4];
      if (same_hi) {
        mms_keep4_hi(hmix, c0, P.thresh, k0);
        mms_keep4_hi(hmix, c0 + 4, P.thresh, k1);
      } else {
        mms_keep4(P.seed, c0, P.thresh, k0);
        mms_keep4(P.seed, c0 + 4, P.thresh, k1);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) { keep[e] = k0[e]; keep[e + 4] = k1[e]; }
    }
    h16x8 o8;
    if (EPI == MMS_EPI_GATE) {
      h16x8 g8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = sigmoidf_(x[e]), ov = (float)ax[pass][e], tv = (float)ax2[pass][e];
        g8[e] = (h16)g;
        o8[e] = (h16)(tv + g * (ov - tv));
      }
      *reinterpret_cast<h16x8*>(P.out2 + (long)m * P.ldo2 + n) = g8;
    } else if (EPI == MMS_EPI_GELU_DROP) {
      h16x8 z8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        z8[e] = (h16)x[e];
        o8[e] = (h16)(keep[e] ? gelu_((float)z8[e]) * dscale : 0.f);
      }
      *reinterpret_cast<h16x8*>(P.out2 + (long)m * P.ldo2 + n) = z8;
    } else if (EPI == MMS_EPI_GELU_DROP_BWD) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o8[e] = (h16)(keep[e] ? x[e] * dscale * gelu_grad_((float)ax[pass][e]) : 0.f);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float o;
        if (EPI == MMS_EPI_RELU_DROP) o = keep[e] ? fmaxf(x[e], 0.f) * dscale : 0.f;
        else if (EPI == MMS_EPI_DROP_RESID) o = (float)ax[pass][e] + (keep[e] ? x[e] * dscale : 0.f);
        else if (EPI == MMS_EPI_RELU_DROP_BWD) o = (float)ax[pass][e] > 0.f ? x[e] * dscale : 0.f;
        else if (EPI == MMS_EPI_F16_ACC) o = (float)ax[pass][e] + x[e];
        else o = x[e];
        o8[e] = (h16)o;
      }
    }
#if defined(MMS_LAB_NOSTORE)   // lab ablation build (scripts/micro): the epilogue without its C stores
    asm volatile("" ::"v"(o8));
#elif defined(MMS_GEMM_NT_STORE)
    __builtin_nontemporal_store(o8, reinterpret_cast<h16x8*>(C + (long)m * P.ldc + n));
#else
    *reinterpret_cast<h16x8*>(C + (long)m * P.ldc + n) = o8;
#endif
  }
}

// ------------------------------------------------------------------------------------------
// BK = 32 variant: 16 KiB stages, a 4-deep ring in the same 64 KiB (2 blocks per CU), so two
// k-tiles stay in flight across every barrier (counted vmcnt, raw s_barrier) instead of one.
// K-contiguous images are [128 rows][32 k] (64-B rows, chunk ^ f(row), f = bits 1,2 of the
// row: conflict-free for ds_read_b128's lane groups); MN-contiguous images are the BK = 64
// layout's first 32 k-rows.
// ------------------------------------------------------------------------------------------
constexpr int BK32 = 32, T32_BYTES = 128 * 32 * 2, ST32 = 4;
MMS_DEV int swz32(int r) { return ((r >> 1) & 1) | (((r >> 2) & 1) << 1); }

template <bool KC>
MMS_DEV h16x8 read_frag32(const char* lds, int sub, int lane) {
  if (KC) {
    const int r = sub + (lane & 15);
    const int c = lane >> 4;
    s16x8 v = *reinterpret_cast<const s16x8*>(lds + r * 64 + ((c ^ swz32(r)) << 4));
    return __builtin_bit_cast(h16x8, v);
  }
  return read_frag<false>(lds, sub, 0, lane);
}

typedef __attribute__((address_space(3))) void lds_void;

// one 128-row x 64-k operand stage by LDS-DMA: 16 wave-instructions, wave `wid` issues 4
template <bool KC>
MMS_DEV void dma_tile(__amdgpu_buffer_rsrc_t rs, char* lds, long ld, int row0, int k0rel, int wid, int lane) {
#ifdef MMS_GEMM_NODMA   // ablation build: no operand traffic (garbage output)
  return;
#endif
  // 16 wave-instructions per 16 KiB tile: wave `wid` issues 4 of them
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ins = wid * 4 + i;
    int voff;
    if (KC) {
      const int row = ins * 8 + (lane >> 3), slot = lane & 7;
      const int c = slot ^ (row & 7);
      voff = (int)(((long)(row0 + row) * ld + k0rel + c * 8) * 2);
    } else {
      const int kr = ins * 4 + (lane >> 4), slot = lane & 15;
      const int c = slot ^ swz_mn(kr);
      voff = (int)(((long)(k0rel + kr) * ld + row0 + c * 8) * 2);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + ins * 1024), 16, voff, 0, 0, 0);
  }
}

template <int N>
MMS_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

#define MMS_EPI_CASES CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_F32) \
    CASE(MMS_EPI_GATE) CASE(MMS_EPI_RELU_DROP_BWD) CASE(MMS_EPI_F16_ACC) CASE(MMS_EPI_GELU_DROP) CASE(MMS_EPI_GELU_DROP_BWD)

}  // namespace
