// Fused multi-head attention (flash-style, online softmax) for the encoder self-attention,
// decoder causal self-attention and decoder cross-attention of mm_s2ut_transformer
// (fairseq MultiheadAttention -> F.multi_head_attention_forward: softmax(q k^T * hd^-0.5 +
// masks) -> dropout -> @ v).  Scores never touch HBM: per (batch, head) a workgroup of 4 waves
// streams 64-key K/V blocks through LDS; each wave owns 16 query rows.
//
// MFMA orientation (v_mfma_f32_16x16x32_f16, D[row][col] with lane l owning col l&15 and rows
// 4(l>>4)+r): the forward computes S^T[key][q] so lane l owns query l&15 and 4 keys per tile;
// exp(S) is converted in registers and fed straight back as the B operand of O^T = V^T P^T,
// with the key order of the two 16-key tiles of a 32-key step permuted identically on the V side
// (two ds_read_b64_tr_b16 at key rows 4g.. and 16+4g..).  Row statistics are lane-local + two
// permlane swaps (lanes l ^ 16, l ^ 32: xmax16_32 / xsum16_32); the O rescale is lane-local.  Dropout on the probabilities uses the same counter
// RNG as the unfused path: counter = offset + (z*Tq + q)*Tk + key.
//
// Backward: D = rowsum(dO*O) (prep kernel); dK/dV with keys stationary (kernel A), dQ with queries
// stationary (kernel B); both recompute P from the saved log-sum-exp — no atomics, deterministic.
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

constexpr int QB = 64, KB = 64;  // streamed query / key rows per LDS tile
constexpr int ATTN_NW = 8;        // waves per block: each owns 16 rows of the block's own dimension

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct AttnP {
  const h16* q; const h16* k; const h16* v; h16* o;
  long ldq, ldk, ldv, ldo;          // row strides (elements)
  long sqb, skb, svb, sob;          // batch strides (elements); head stride = hd
  int H, Tq, Tk;
  const int* key_len;               // [B] or null
  int causal;
  float scale;
  float p; uint32_t thresh; uint64_t seed, offset;
  float* lse;                       // [Z*Tq]
  // backward
  const h16* dout; long lddo, sdob;
  const float* Dd;                  // [Z*Tq] rowsum(dO*O)
  h16* dq; h16* dk; h16* dv;
  long lddq, lddk, lddv, sdqb, sdkb, sdvb;
  int kv16;                         // dK / dV rows 16-B aligned: the fused backward stores 16 B per lane
};

template <int HD>
struct Tile {
  // padded LDS row (halves).  HD + 16 (a row stride of 8 dwords mod 16): the 16-lane groups that
  // gfx950 services per ds_read_b128 cycle ({0-3,12-15,20-27}, ...: rows 0-3 and 12-15 of one
  // 8-half column block with rows 4-11 of the next) and the 32-lane groups of ds_read_b64_tr_b16
  // then touch every bank once; HD + 8 (round 1-4) conflicted 2-way on both reads
  // (SQ_LDS_BANK_CONFLICT 1.6x the LDS-active cycles of the fused backward, round-5 PMC)
  static constexpr int LD = HD + 16;
  static constexpr int CH = HD / 8;  // 16-B chunks per row
};

// Register-staged prefetch of a pair of 64-row tiles (K/V or Q/dO): every global load of the
// pair is issued at once and only stored to LDS at the top of the next iteration, so the load
// latency hides behind the current tile's MFMAs (load-then-store per chunk serialised ~2 us of
// latency per chunk round).  Optionally carries two fp32 per row (LSE, D) for the first 64 lanes.
template <int HD, int NT>
struct Pair64 {
  static constexpr int CH = HD / 8, LD = Tile<HD>::LD;
  static constexpr int N = (64 * CH + NT - 1) / NT;
  s16x8 a[N], b[N];
  float fl, fd;
  MMS_DEV void load(const h16* ga, long lda, const h16* gb, long ldb, int row0, int valid) {
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const int i = threadIdx.x + n * NT;
      const int r = i / CH, c = i % CH;
      const s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      a[n] = z;
      b[n] = z;
      if (i < 64 * CH && row0 + r < valid) {
        a[n] = *reinterpret_cast<const s16x8*>(ga + (long)(row0 + r) * lda + c * 8);
        b[n] = *reinterpret_cast<const s16x8*>(gb + (long)(row0 + r) * ldb + c * 8);
      }
    }
  }
  MMS_DEV void load_stats(const float* L, const float* D, long base, int row0, int valid) {
    const int i = threadIdx.x;
    fl = fd = 0.f;
    if (i < 64 && row0 + i < valid) {
      fl = L[base + row0 + i];
      fd = D[base + row0 + i];
    }
  }
  MMS_DEV void store(h16* la, h16* lb) const {
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const int i = threadIdx.x + n * NT;
      const int r = i / CH, c = i % CH;
      if (i < 64 * CH) {
        *reinterpret_cast<s16x8*>(la + r * LD + c * 8) = a[n];
        *reinterpret_cast<s16x8*>(lb + r * LD + c * 8) = b[n];
      }
    }
  }
};

// A/B fragment with rows along LDS rows: lane l -> X[row0 + (l&15)][k0 + 8(l>>4) .. +7]
template <int HD>
MMS_DEV h16x8 frag_rows(const h16* lds, int row0, int k0, int lane) {
  const h16* p = lds + (row0 + (lane & 15)) * Tile<HD>::LD + k0 + 8 * (lane >> 4);
  return __builtin_bit_cast(h16x8, *reinterpret_cast<const s16x8*>(p));
}

// transposed fragment over a 32-row step with the (4g.., 16+4g..) row permutation:
// lane l (group g, i = l&15) -> X[row0 + 4g + j][col0 + i] (j<4), X[row0 + 16 + 4g + j-4][col0 + i]
template <int LDX>
MMS_DEV h16x8 frag_tr_ld(const h16* lds, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const h16* a1 = lds + (row0 + 4 * g + q) * LDX + col0 + 4 * pp;
  const h16* a2 = a1 + 16 * LDX;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a2));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(h16x8, v);
}

template <int HD>
MMS_DEV h16x8 frag_tr(const h16* lds, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const h16* a1 = lds + (row0 + 4 * g + q) * Tile<HD>::LD + col0 + 4 * pp;
  const h16* a2 = a1 + 16 * Tile<HD>::LD;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a2));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(h16x8, v);
}

// buffer resource over `rows` rows of stride ld (elements) from base: loads of rows >= rows (or
// rows <= 0) are out of range and return zero
MMS_DEV __amdgpu_buffer_rsrc_t rsrc_rows(const h16* base, int rows, long ld) {
  const int bytes = rows > 0 ? (int)(rows * ld * 2) : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
MMS_DEV s16x8 ld16b(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

// key length of batch row b (b wave-uniform) through the scalar cache: a vector load here would
// share vmcnt with the register prefetches in flight, and waiting for it (the value feeds buffer
// descriptors and loop bounds at once) would drain them all
MMS_DEV int key_len_of(const AttnP& P, int b) {
  if (!P.key_len) return P.Tk;
  typedef const __attribute__((address_space(4))) int cint4;
  const int v = ((cint4*)(unsigned long)P.key_len)[b];
  return min(v, P.Tk);
}
MMS_DEV f32x4 mfma(h16x8 a, h16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

MMS_DEV h16x8 pack8(f32x4 a, f32x4 b) {
  return h16x8{(h16)a[0], (h16)a[1], (h16)a[2], (h16)a[3], (h16)b[0], (h16)b[1], (h16)b[2], (h16)b[3]};
}

// over the four lanes l, l ^ 16, l ^ 32, l ^ 48 (one query row's 4 key groups): permlane swaps,
// no LDS round trip
MMS_DEV float xmax16_32(float v) { return xmax32(xmax16(v)); }
MMS_DEV float xsum16_32(float v) { return xsum32(xsum16(v)); }

#ifdef MMS_ATTN_PHASES
// diagnostic build only (scripts/attn_phases.py): s_memtime at the phase boundaries of the first
// blocks' first chunks, read back with mms2ut_diag_attn_phases
__device__ unsigned long long g_attn_ph[64 * 64];
#define PH_STAMP(slot)                                                                          \
  do {                                                                                          \
    if (ph_blk < 64 && tid == 0 && (slot) < 64) g_attn_ph[ph_blk * 64 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define PH_STAMP(slot) do { } while (0)
#endif

// ============================================================================ forward
// SHORT (Tk <= 128): the head's whole K / V (<= 2 tiles) is loaded into LDS in one burst up front
// — one load latency per block instead of one per 64-key tile — and the tile loop runs without
// barriers.
template <int HD, int NW, bool SHORT = false>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4))) attn_fwd_kernel(AttnP P) {
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  constexpr int OWN = 16 * NW;  // query rows owned by the block (16 per wave)
  constexpr int LD = Tile<HD>::LD, NKK = HD / 32, NDT = HD / 16;
  constexpr int KROWS = SHORT ? 2 * KB : KB;
  __shared__ __attribute__((aligned(16))) h16 sK[KROWS * LD];
  __shared__ __attribute__((aligned(16))) h16 sV[KROWS * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int z = blockIdx.y, b = z / P.H, h = z % P.H;
  const int qblk = blockIdx.x * OWN;
  const int w_row0 = qblk + w * 16, q_own = w_row0 + (lane & 15);  // this lane's query row
  const int klen = key_len_of(P, b);
  int kmax = klen;
  if (P.causal) kmax = min(kmax, qblk + OWN);
  const h16* Q = P.q + b * P.sqb + h * HD;
  const h16* K = P.k + b * P.skb + h * HD;
  const h16* V = P.v + b * P.svb + h * HD;
  const int tid = threadIdx.x, ph_blk = blockIdx.y * gridDim.x + blockIdx.x;
  (void)tid; (void)ph_blk;
  PH_STAMP(0);
  // Q^T fragments (B operand): lane -> Q[q_own][kk*32 + 8g .. +7]
  h16x8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    s16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q_own < P.Tq) t = *reinterpret_cast<const s16x8*>(Q + (long)q_own * P.ldq + kk * 32 + 8 * g);
    qf[kk] = __builtin_bit_cast(h16x8, t);
  }
  f32x4 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;   // running max of the unscaled scores, running sum
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  const float c2 = P.scale * 1.4426950408889634f;   // scale * log2(e)
  const uint64_t row_ctr = P.offset + ((uint64_t)z * P.Tq + q_own) * (uint64_t)P.Tk;
  const uint64_t zctr = P.offset + (uint64_t)z * P.Tq * P.Tk;
  const bool hi_fast = mms_same_hi(zctr, zctr + (uint64_t)P.Tq * P.Tk - 1);  // uniform per head
  // every row's counters start even (even base, even key length): a key quad's two hash pairs are
  // pair indices prow + (key >> 1) + {0, 1}, in 32-bit arithmetic (bit-identical to mms_keep4_hi)
  const bool hi_pairs = hi_fast && (zctr & 1) == 0 && (P.Tk & 1) == 0;
  const uint32_t prow = (uint32_t)(row_ctr >> 1);
  const uint32_t hi_mix = mms_hi_mix(P.seed, zctr);
  Pair64<HD, 64 * NW> pf;
  if constexpr (SHORT) {
    constexpr int CH = HD / 8, NLS = (KROWS * CH + 64 * NW - 1) / (64 * NW);
    const auto rK = rsrc_rows(K, kmax, P.ldk);
    const auto rV = rsrc_rows(V, kmax, P.ldv);
    s16x8 rk[NLS], rv[NLS];
#pragma unroll
    for (int n = 0; n < NLS; ++n) {
      const int i = threadIdx.x + n * 64 * NW, r = i / CH, c = i % CH;
      if ((KROWS * CH) % (64 * NW) == 0 || i < KROWS * CH) {
        rk[n] = ld16b(rK, (r * (int)P.ldk + c * 8) * 2);  // rows >= kmax read as zero
        rv[n] = ld16b(rV, (r * (int)P.ldv + c * 8) * 2);
      }
    }
#pragma unroll
    for (int n = 0; n < NLS; ++n) {
      const int i = threadIdx.x + n * 64 * NW, r = i / CH, c = i % CH;
      if ((KROWS * CH) % (64 * NW) == 0 || i < KROWS * CH) {
        *reinterpret_cast<s16x8*>(sK + r * LD + c * 8) = rk[n];
        *reinterpret_cast<s16x8*>(sV + r * LD + c * 8) = rv[n];
      }
    }
    __syncthreads();
  } else {
    if (kmax > 0) pf.load(K, P.ldk, V, P.ldv, 0, kmax);
  }
  PH_STAMP(1);
  for (int kb = 0; kb < kmax; kb += KB) {
    PH_STAMP(2 + 2 * (kb / KB));
    const h16* tK = SHORT ? sK + kb * LD : sK;
    const h16* tV = SHORT ? sV + kb * LD : sV;
    if constexpr (!SHORT) {
      __syncthreads();
      pf.store(sK, sV);
      // every load issued so far has landed (the stores above waited for the tile's): re-define the
      // Q fragments here, or the compiler -- unable to prove across the loop that their loads are
      // done -- puts vmcnt(0) in front of the first QK^T MFMA, draining the next tile's prefetch
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(qf[kk]));
      __syncthreads();
      if (kb + KB < kmax) pf.load(K, P.ldk, V, P.ldv, kb + KB, kmax);
    }
    PH_STAMP(3 + 2 * (kb / KB));
    // a wave past the last query row, or whose rows all precede this key tile (causal), only
    // helps stage K/V
    if (w_row0 >= P.Tq || (P.causal && kb > w_row0 + 15)) continue;
    // S^T for 4 tiles of 16 keys: lane -> S[q_own][kb + 16t + 4g + r]
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) s[t] = mfma(frag_rows<HD>(tK, 16 * t, kk * 32, lane), qf[kk], s[t]);
    }
    // scores stay unscaled: the max commutes with the positive scale, and exp(scale*(s - m)) is one
    // FMA + v_exp_f32 in base 2.  A key tile that is valid for every row of the wave (inside the
    // key length and, causal, entirely at or before the wave's first row) skips the masking.
    const bool full = kb + KB <= kmax && (!P.causal || kb + KB - 1 <= w_row0);
    float bmax = -INFINITY;
    if (full) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
        bmax = fmaxf(bmax, fmaxf(fmaxf(s[t][0], s[t][1]), fmaxf(s[t][2], s[t][3])));
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb + 16 * t + 4 * g + r;
          const bool ok = key < kmax && (!P.causal || key <= q_own);
          const float x = ok ? s[t][r] : -INFINITY;
          s[t][r] = x;
          bmax = fmaxf(bmax, x);
        }
    }
    bmax = xmax16_32(bmax);
    const float mn = fmaxf(m, bmax);
    const float alpha = (mn == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f((m - mn) * c2);
    const float mnc = (mn == -INFINITY) ? 0.f : mn * c2;   // masked s = -inf -> exp2(-inf) = 0
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bool keep[4] = {true, true, true, true};
      if (P.thresh) {
        if (hi_pairs) {
          const uint32_t p0 = prow + (uint32_t)((kb + 16 * t + 4 * g) >> 1);
          const uint32_t h0 = mms_mix32(p0 ^ hi_mix), h1 = mms_mix32((p0 + 1) ^ hi_mix);
          keep[0] = (h0 & 0xffffU) >= P.thresh;
          keep[1] = (h0 >> 16) >= P.thresh;
          keep[2] = (h1 & 0xffffU) >= P.thresh;
          keep[3] = (h1 >> 16) >= P.thresh;
        } else if (hi_fast) {
          mms_keep4_hi(hi_mix, row_ctr + kb + 16 * t + 4 * g, P.thresh, keep);
        } else {
          mms_keep4(P.seed, row_ctr + kb + 16 * t + 4 * g, P.thresh, keep);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __builtin_amdgcn_exp2f(fmaf(s[t][r], c2, -mnc));
        rs += e;
        s[t][r] = keep[r] ? e : 0.f;   // the 1/(1-p) of the kept probabilities is applied once at the end
      }
    }
    rs = xsum16_32(rs);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[i] *= alpha;
    // O^T[d][q] += V^T[d][keys] P^T[keys][q], two 32-key steps
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const h16x8 pf = pack8(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int i = 0; i < NDT; ++i) o[i] = mfma(frag_tr<HD>(tV, 32 * c, 16 * i, lane), pf, o[i]);
    }
  }
  PH_STAMP(40);
  if (q_own < P.Tq) {
    const float inv = l > 0.f ? dscale / l : 0.f;
    h16* O = P.o + b * P.sob + h * HD + (long)q_own * P.ldo;
#pragma unroll
    for (int i = 0; i < NDT; ++i)
      *reinterpret_cast<h16x4*>(O + 16 * i + 4 * g) =
          h16x4{(h16)(o[i][0] * inv), (h16)(o[i][1] * inv), (h16)(o[i][2] * inv), (h16)(o[i][3] * inv)};
    // natural-log LSE of the scaled scores (the backward's exp(s*scale - L))
    if (g == 0 && P.lse) P.lse[(long)z * P.Tq + q_own] = (l > 0.f) ? m * P.scale + __logf(l) : -INFINITY;
  }
  PH_STAMP(41);
}

// ============================================================================ backward prep
template <int HD>
__global__ void attn_bwd_prep_kernel(AttnP P, int Z) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)Z * P.Tq) return;
  const int z = (int)(row / P.Tq), t = (int)(row % P.Tq);
  const int b = z / P.H, h = z % P.H;
  const h16* O = P.o + b * P.sob + h * HD + (long)t * P.ldo;
  const h16* dO = P.dout + b * P.sdob + h * HD + (long)t * P.lddo;
  float s = 0.f;
  for (int d = lane * 2; d < HD; d += 128) {
    s += (float)O[d] * (float)dO[d];
    if (d + 1 < HD) s += (float)O[d + 1] * (float)dO[d + 1];
  }
  s = wave_sum(s);
  if (lane == 0) const_cast<float*>(P.Dd)[row] = s;
}

// One wave per token row covering every head: lane = h * (64/H) + j reads chunks j, j + 64/H, ...
// (4 halfs each) of head h, then a (64/H)-lane segmented reduction.  Needs 64 % H == 0 and
// (HD/4) % (64/H) == 0 (host check); 8-B loads, whole rows per wave instruction group.
template <int HD>
__global__ void __launch_bounds__(256) attn_bwd_prep_rows_kernel(AttnP P, long nrows) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const int b = (int)(row / P.Tq), t = (int)(row % P.Tq);
  const int LPH = 64 / P.H;               // lanes per head
  const int h = lane / LPH, j = lane % LPH;
  const h16* O = P.o + b * P.sob + (long)t * P.ldo + h * HD;
  const h16* dO = P.dout + b * P.sdob + (long)t * P.lddo + h * HD;
  float s = 0.f;
  for (int c = j; c < HD / 4; c += LPH) {
    const h16x4 o = *reinterpret_cast<const h16x4*>(O + 4 * c);
    const h16x4 d = *reinterpret_cast<const h16x4*>(dO + 4 * c);
#pragma unroll
    for (int e = 0; e < 4; ++e) s += (float)o[e] * (float)d[e];
  }
  for (int off = LPH >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (j == 0) const_cast<float*>(P.Dd)[((long)b * P.H + h) * P.Tq + t] = s;
}

// ============================================================================ backward: dK, dV
template <int HD, int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_kv_kernel(AttnP P) {
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  constexpr int OWN = 16 * NW;  // keys owned by the block
  constexpr int LD = Tile<HD>::LD, NKK = HD / 32, NDT = HD / 16;
  __shared__ __attribute__((aligned(16))) h16 sQ[QB * LD];
  __shared__ __attribute__((aligned(16))) h16 sDO[QB * LD];
  __shared__ float sL[QB], sD[QB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int z = blockIdx.y, b = z / P.H, h = z % P.H;
  const int kblk = blockIdx.x * OWN;
  const int key_own = kblk + w * 16 + (lane & 15);
  const int klen = key_len_of(P, b);
  const h16* Q = P.q + b * P.sqb + h * HD;
  const h16* K = P.k + b * P.skb + h * HD;
  const h16* V = P.v + b * P.svb + h * HD;
  const h16* DO = P.dout + b * P.sdob + h * HD;
  // K^T, V^T fragments of this wave's 16 keys (B operands): lane -> X[key_own][kk*32 + 8g ..]
  h16x8 kf[NKK], vf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    s16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = a;
    if (key_own < klen) {
      a = *reinterpret_cast<const s16x8*>(K + (long)key_own * P.ldk + kk * 32 + 8 * g);
      c = *reinterpret_cast<const s16x8*>(V + (long)key_own * P.ldv + kk * 32 + 8 * g);
    }
    kf[kk] = __builtin_bit_cast(h16x8, a);
    vf[kk] = __builtin_bit_cast(h16x8, c);
  }
  f32x4 dk[NDT], dv[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) { dk[i] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[i] = dk[i]; }
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  const int q_begin = P.causal ? (kblk / QB) * QB : 0;
  if (kblk < klen) {
    Pair64<HD, 64 * NW> pf;
    if (q_begin < P.Tq) {
      pf.load(Q, P.ldq, DO, P.lddo, q_begin, P.Tq);
      pf.load_stats(P.lse, P.Dd, (long)z * P.Tq, q_begin, P.Tq);
    }
    for (int qb = q_begin; qb < P.Tq; qb += QB) {
      __syncthreads();
      pf.store(sQ, sDO);
      if (threadIdx.x < QB) {
        sL[threadIdx.x] = pf.fl;
        sD[threadIdx.x] = pf.fd;
      }
      __syncthreads();
      if (qb + QB < P.Tq) {
        pf.load(Q, P.ldq, DO, P.lddo, qb + QB, P.Tq);
        pf.load_stats(P.lse, P.Dd, (long)z * P.Tq, qb + QB, P.Tq);
      }
      // per 16-query tile: S[q][key], dP'[q][key]; lane -> (q = qb + 16t + 4g + r, key_own)
      f32x4 pt[4], dst[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = s;
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          s = mfma(frag_rows<HD>(sQ, 16 * t, kk * 32, lane), kf[kk], s);
          dp = mfma(frag_rows<HD>(sDO, 16 * t, kk * 32, lane), vf[kk], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = 16 * t + 4 * g + r, q = qb + qi;
          const bool ok = q < P.Tq && key_own < klen && (!P.causal || key_own <= q);
          const float pr = ok ? __expf(s[r] * P.scale - sL[qi]) : 0.f;
          float mk = dscale;
          if (P.thresh && ok)
            mk = mms_keep(P.seed, P.offset + ((uint64_t)z * P.Tq + q) * (uint64_t)P.Tk + key_own, P.thresh) ? dscale : 0.f;
          pt[t][r] = pr * mk;                              // P' (dropped)
          dst[t][r] = pr * (dp[r] * mk - sD[qi]);          // dS
        }
      }
      // dV^T[d][key] += dO^T[d][q] P'[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const h16x8 pf = pack8(pt[2 * c], pt[2 * c + 1]);
        const h16x8 sf = pack8(dst[2 * c], dst[2 * c + 1]);
#pragma unroll
        for (int i = 0; i < NDT; ++i) {
          dv[i] = mfma(frag_tr<HD>(sDO, 32 * c, 16 * i, lane), pf, dv[i]);
          dk[i] = mfma(frag_tr<HD>(sQ, 32 * c, 16 * i, lane), sf, dk[i]);
        }
      }
    }
  }
  if (key_own < P.Tk) {
    h16* DK = P.dk + b * P.sdkb + h * HD + (long)key_own * P.lddk;
    h16* DV = P.dv + b * P.sdvb + h * HD + (long)key_own * P.lddv;
#pragma unroll
    for (int i = 0; i < NDT; ++i) {
      const f32x4 a = dk[i] * P.scale, c = dv[i];
      *reinterpret_cast<h16x4*>(DK + 16 * i + 4 * g) = h16x4{(h16)a[0], (h16)a[1], (h16)a[2], (h16)a[3]};
      *reinterpret_cast<h16x4*>(DV + 16 * i + 4 * g) = h16x4{(h16)c[0], (h16)c[1], (h16)c[2], (h16)c[3]};
    }
  }
}

// ============================================================================ backward: dQ
template <int HD, int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_q_kernel(AttnP P) {
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  constexpr int OWN = 16 * NW;
  constexpr int LD = Tile<HD>::LD, NKK = HD / 32, NDT = HD / 16;
  __shared__ __attribute__((aligned(16))) h16 sK[KB * LD];
  __shared__ __attribute__((aligned(16))) h16 sV[KB * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int z = blockIdx.y, b = z / P.H, h = z % P.H;
  const int qblk = blockIdx.x * OWN;
  const int q_own = qblk + w * 16 + (lane & 15);
  const int klen = key_len_of(P, b);
  int kmax = klen;
  if (P.causal) kmax = min(kmax, qblk + OWN);
  const h16* Q = P.q + b * P.sqb + h * HD;
  const h16* K = P.k + b * P.skb + h * HD;
  const h16* V = P.v + b * P.svb + h * HD;
  const h16* DO = P.dout + b * P.sdob + h * HD;
  const bool qok = q_own < P.Tq;
  h16x8 qf[NKK], df[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    s16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = a;
    if (qok) {
      a = *reinterpret_cast<const s16x8*>(Q + (long)q_own * P.ldq + kk * 32 + 8 * g);
      c = *reinterpret_cast<const s16x8*>(DO + (long)q_own * P.lddo + kk * 32 + 8 * g);
    }
    qf[kk] = __builtin_bit_cast(h16x8, a);
    df[kk] = __builtin_bit_cast(h16x8, c);
  }
  const float L = qok ? P.lse[(long)z * P.Tq + q_own] : 0.f;
  const float Dq = qok ? P.Dd[(long)z * P.Tq + q_own] : 0.f;
  f32x4 dq[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  const uint64_t row_ctr = P.offset + ((uint64_t)z * P.Tq + q_own) * (uint64_t)P.Tk;
  const uint64_t zctr = P.offset + (uint64_t)z * P.Tq * P.Tk;
  const bool hi_fast = mms_same_hi(zctr, zctr + (uint64_t)P.Tq * P.Tk - 1);  // uniform per head
  const uint32_t hi_mix = mms_hi_mix(P.seed, zctr);
  Pair64<HD, 64 * NW> pf;
  if (kmax > 0) pf.load(K, P.ldk, V, P.ldv, 0, kmax);
  for (int kb = 0; kb < kmax; kb += KB) {
    __syncthreads();
    pf.store(sK, sV);
    __syncthreads();
    if (kb + KB < kmax) pf.load(K, P.ldk, V, P.ldv, kb + KB, kmax);
    f32x4 ds[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = s;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        s = mfma(frag_rows<HD>(sK, 16 * t, kk * 32, lane), qf[kk], s);
        dp = mfma(frag_rows<HD>(sV, 16 * t, kk * 32, lane), df[kk], dp);
      }
      bool keep[4] = {true, true, true, true};
      if (P.thresh) {
        if (hi_fast) mms_keep4_hi(hi_mix, row_ctr + kb + 16 * t + 4 * g, P.thresh, keep);
        else mms_keep4(P.seed, row_ctr + kb + 16 * t + 4 * g, P.thresh, keep);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb + 16 * t + 4 * g + r;
        const bool ok = qok && key < kmax && (!P.causal || key <= q_own);
        const float pr = ok ? __expf(s[r] * P.scale - L) : 0.f;
        const float mk = keep[r] ? dscale : 0.f;
        ds[t][r] = pr * (dp[r] * mk - Dq);
      }
    }
    // dQ^T[d][q] += K^T[d][keys] dS^T[keys][q]
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const h16x8 sf = pack8(ds[2 * c], ds[2 * c + 1]);
#pragma unroll
      for (int i = 0; i < NDT; ++i) dq[i] = mfma(frag_tr<HD>(sK, 32 * c, 16 * i, lane), sf, dq[i]);
    }
  }
  if (qok) {
    h16* DQ = P.dq + b * P.sdqb + h * HD + (long)q_own * P.lddq;
#pragma unroll
    for (int i = 0; i < NDT; ++i) {
      const f32x4 a = dq[i] * P.scale;
      *reinterpret_cast<h16x4*>(DQ + 16 * i + 4 * g) = h16x4{(h16)a[0], (h16)a[1], (h16)a[2], (h16)a[3]};
    }
  }
}


// ============================================================================ backward: fused, Tk <= 256
// One workgroup per (b, h) when Tk <= 256 (every length of the step's encoder / decoder / cross
// attention): the head's K stays in LDS, each wave keeps V fragments of its own keys in registers,
// and the queries stream through in chunks of QC rows.  Per chunk: phase 2 (keys stationary)
// accumulates dK/dV in registers across all chunks and writes dS^T [key][query] to LDS; phase 3
// (queries stationary) forms dQ = dS K for the chunk from LDS.  D = rowsum(dO*O) is formed while
// the chunk is stored; the next chunk's Q/dO/O rows are loaded into registers during the current
// chunk's MFMA phases.  No prep launch, no second pass that re-reads Q/K/V/dO and recomputes P.
//   NKC = key chunks of 128 (1 or 2): wave w owns keys 16w + 128j (j < NKC); QC = 128 / NKC.
template <int HD, int NKC>
struct FusedCfg {
  static constexpr int QC = 128 / NKC, TKP = 128 * NKC, LDS_T = QC + 8;
  static constexpr int NQT = QC / 16, DSPLIT = 8 / NQT;
  static constexpr int CH = HD / 8, NLQ = (QC * CH + 511) / 512, NLK = (TKP * CH + 511) / 512;
};


template <int HD, int NKC>
__global__ void __launch_bounds__(512) attn_bwd_fused_kernel(AttnP P, int Z) {
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  using F = FusedCfg<HD, NKC>;
  constexpr int LD = Tile<HD>::LD, NKK = HD / 32, NDT = HD / 16, CH = F::CH;
  constexpr int QC = F::QC, TKP = F::TKP, LDS_T = F::LDS_T, NQT = F::NQT, NDW = NDT / F::DSPLIT;
  constexpr int NLQ = F::NLQ, NLK = F::NLK;
  static_assert(NDT % F::DSPLIT == 0, "d tiles must split evenly over the phase-3 wave pairs");
  __shared__ __attribute__((aligned(16))) h16 sK[TKP * LD];
  __shared__ __attribute__((aligned(16))) h16 sQ[QC * LD];
  __shared__ __attribute__((aligned(16))) h16 sDO[QC * LD];
  __shared__ __attribute__((aligned(16))) h16 sDS[TKP * LDS_T];  // dS^T [key][query of the chunk]
  __shared__ __attribute__((aligned(16))) float sL[2][QC];
  __shared__ __attribute__((aligned(16))) float sD[2][QC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int Tq = P.Tq, nch = (Tq + QC - 1) / QC;
  const s16x8 zz = {0, 0, 0, 0, 0, 0, 0, 0};
  const float dscale = P.thresh ? 1.f / (1.f - P.p) : 1.f;
  const float c2 = P.scale * 1.4426950408889634f;   // scale * log2(e); sL holds the LSE * log2(e)
  // register staging: the rows of one query chunk, K of one head, V fragments of the wave's keys
  s16x8 rq[NLQ], rd[NLQ], ro[NLQ], rk[NLK];
  float rl = 0.f;
  h16x8 vf[NKC][NKK];
  // Loads go through buffer resources built per head / chunk (SGPRs): rows past the valid range
  // fall outside num_records and read as zero, and the per-thread offsets stay 32-bit.
  auto load_chunk = [&](int zc, int qbase) {
    int tid_ = tid;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_;
    const int bc = zc / P.H, hc = zc % P.H, rows = Tq - qbase;
    const auto rQ = rsrc_rows(P.q + bc * P.sqb + hc * HD + (long)qbase * P.ldq, rows, P.ldq);
    const auto rD = rsrc_rows(P.dout + bc * P.sdob + hc * HD + (long)qbase * P.lddo, rows, P.lddo);
    const auto rO = rsrc_rows(P.o + bc * P.sob + hc * HD + (long)qbase * P.ldo, rows, P.ldo);
#pragma unroll
    for (int n = 0; n < NLQ; ++n) {
      const int i = tid + n * 512, r = i / CH, c = i % CH;
      if (QC * CH % 512 == 0 || i < QC * CH) {  // straight-line when every thread loads
        rq[n] = ld16b(rQ, (r * (int)P.ldq + c * 8) * 2);
        rd[n] = ld16b(rD, (r * (int)P.lddo + c * 8) * 2);
        ro[n] = ld16b(rO, (r * (int)P.ldo + c * 8) * 2);
      }
    }
    // LSE of the chunk's rows (threads >= QC load a value nobody reads; rows >= Tq read 0)
    const __amdgpu_buffer_rsrc_t rL = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(P.lse + (long)zc * Tq + qbase), (short)0, rows > 0 ? rows * 4 : 0, 0x00020000);
    rl = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rL, tid * 4, 0, 0));
  };
  // live = false: the same load instructions over an empty range (they return zeros without
  // touching memory) -- see the LAST chunk below
  auto load_kv = [&](int zc, bool live) {
    int tid_ = tid;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_, lane = tid & 63, g = lane >> 4, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bc = zc / P.H, hc = zc % P.H;
    const int kl = live ? key_len_of(P, bc) : 0;
    const auto rK = rsrc_rows(P.k + bc * P.skb + hc * HD, kl, P.ldk);
    const auto rV = rsrc_rows(P.v + bc * P.svb + hc * HD, kl, P.ldv);
#pragma unroll
    for (int n = 0; n < NLK; ++n) {
      const int i = tid + n * 512, r = i / CH, c = i % CH;
      if (TKP * CH % 512 == 0 || i < TKP * CH) rk[n] = ld16b(rK, (r * (int)P.ldk + c * 8) * 2);
    }
#pragma unroll
    for (int j = 0; j < NKC; ++j) {
      const int key = 16 * w + 128 * j + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
        vf[j][kk] = __builtin_bit_cast(h16x8, ld16b(rV, (key * (int)P.ldv + kk * 32 + 8 * g) * 2));
    }
  };
  // persistent: block i handles the heads of a snake order over rounds of G = gridDim.x heads --
  // i, 2G - 1 - i, 2G + i, 4G - 1 - i, ... -- so the blocks that take a head of the last, partial
  // round took a shorter one in the round before (heads come in batch-row order, and the collater
  // sorts rows by length); the next head's rows, K and V are loaded into registers while the
  // current head's MFMA phases run.  Once a block's next head is past Z, every later one is too.
  const int G = gridDim.x, bid = blockIdx.x;
  auto head_at = [&](int k) { return (k & 1) ? (k + 1) * G - 1 - bid : k * G + bid; };
  int hk = 0;
  int z = blockIdx.x;
  if (z >= Z) return;
  const int ph_blk = blockIdx.x;
  (void)ph_blk;
  PH_STAMP(0);
  load_chunk(z, 0);
  load_kv(z, true);
  static_assert(QC * CH * sizeof(float) <= sizeof(sDS), "D partials must fit the dS^T buffer");
  int gc = 0;  // running chunk counter: parity selects the sL / sD buffer
  for (; z < Z; z = head_at(++hk)) {
    const int b = z / P.H, h = z % P.H, znext = head_at(hk + 1);
    const int klen = key_len_of(P, b);
    __syncthreads();  // the previous head's phase 3 is done with sK
#pragma unroll
    for (int n = 0; n < NLK; ++n) {
      const int i = tid + n * 512, r = i / CH, c = i % CH;
      if (i < TKP * CH) *reinterpret_cast<s16x8*>(sK + r * LD + c * 8) = rk[n];
    }
    // vf arrived with rk (same load_kv), which the stores above have waited for; re-define vf here
    // so the compiler's wait tracking, which loses count across the head loop, does not put
    // vmcnt(1..3) waits (draining the next chunk's prefetch) in front of phase 2's dV MFMAs
#pragma unroll
    for (int j = 0; j < NKC; ++j)
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(vf[j][kk]));
    f32x4 dk[NKC][NDT], dv[NKC][NDT];
#pragma unroll
    for (int j = 0; j < NKC; ++j)
#pragma unroll
      for (int i = 0; i < NDT; ++i) { dk[j][i] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[j][i] = dk[j][i]; }
    // one query chunk; the last chunk of the head also writes dK / dV and prefetches the next head
    // (peeled, so that the next head's K stays out of the register live range of phase 2)
    auto chunk = [&](const int ch, auto last_c) {
      constexpr bool LAST = decltype(last_c)::value;
      // per-thread indices re-derived from an opaque copy of tid: keeps the compiler from hoisting
      // dozens of per-lane offsets / counters out of the head loop (they would spill)
      int tl = tid;
      asm volatile("" : "+v"(tl));
      const int lane = tl & 63, g = lane >> 4, w = __builtin_amdgcn_readfirstlane(tl >> 6);
      const int qbase = ch * QC, buf = gc & 1;
      float* L = sL[buf];
      float* Dr = sD[buf];
      const uint64_t zctr = P.offset + (uint64_t)z * Tq * (uint64_t)P.Tk;  // RNG counter of (z, 0, 0)
      const bool hi_fast = mms_same_hi(zctr, zctr + (uint64_t)Tq * P.Tk - 1);  // uniform
      // every row's counters start even (even base, even key length): key pairs 2m, 2m+1 share a hash
      const bool hi_pairs = hi_fast && (zctr & 1) == 0 && (P.Tk & 1) == 0;
      const uint32_t hi_mix = mms_hi_mix(P.seed, zctr);
      // ---- phase 1: staged rows -> LDS, D = rowsum(dO*O); prefetch the next chunk / head
      PH_STAMP(1 + 5 * gc);
      __syncthreads();  // previous chunk's phase 3 is done with sDS, its phase 2 with sQ / sDO
      PH_STAMP(2 + 5 * gc);
#pragma unroll
      for (int n = 0; n < NLQ; ++n) {
        const int i = tid + n * 512, r = i / CH, c = i % CH;
        if (i < QC * CH) {
          *reinterpret_cast<s16x8*>(sQ + r * LD + c * 8) = rq[n];
          *reinterpret_cast<s16x8*>(sDO + r * LD + c * 8) = rd[n];
          const h16x8 o8 = __builtin_bit_cast(h16x8, ro[n]), d8 = __builtin_bit_cast(h16x8, rd[n]);
          float dot = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) dot += (float)o8[e] * (float)d8[e];
          // row r's CH partial dots go to sDS (free until phase 2) at [r][c] = i, summed below in
          // column order: deterministic (no LDS float atomics)
          reinterpret_cast<float*>(sDS)[i] = (qbase + r < Tq) ? dot : 0.f;
        }
      }
      if (tid < QC) L[tid] = rl * 1.4426950408889634f;   // LSE in log2 units
      // The prefetch is issued unconditionally (past the last head: an empty row range, so the
      // loads return zeros without touching memory).  A conditional issue leaves the compiler
      // unsure how many loads are in flight, and it then waits for all of them (vmcnt(0)) at the
      // first MFMA of phase 2 -- exposing the next head's load latency on every head's last chunk.
      if (!LAST) load_chunk(z, qbase + QC);
      else load_chunk(znext < Z ? znext : z, znext < Z ? 0 : Tq);
      __syncthreads();
      if (tid < QC) {
        const float* part = reinterpret_cast<const float*>(sDS) + tid * CH;
        float dsum = 0.f;
#pragma unroll
        for (int c = 0; c < CH; ++c) dsum += part[c];
        Dr[tid] = dsum;
      }
      __syncthreads();   // D complete; phase 2 overwrites sDS
      PH_STAMP(3 + 5 * gc);
      // ---- phase 2: wave w owns keys 16w + 128j: dV, dK accumulate, dS^T -> LDS.  Query steps
      // outermost: the step's Q / dO row fragments and the transposed dO / Q operands of the dV / dK
      // MFMAs are read from LDS once and used for all NKC key groups of the wave (half the LDS
      // reads of a key-group-outer loop at NKC = 2); values and rounding points are unchanged.
      for (int qs = 0; qs < QC; qs += 32) {
        const int qa = qbase + qs;
        bool act[NKC];
        bool any = false;
#pragma unroll
        for (int j = 0; j < NKC; ++j) {
          const int kw0 = 16 * w + 128 * j, key_own = kw0 + (lane & 15);
          act[j] = !(kw0 >= klen || qa >= Tq || (P.causal && qa + 31 < kw0));   // wave-uniform
          any = any || act[j];
          if (!act[j]) {
            *reinterpret_cast<h16x4*>(sDS + key_own * LDS_T + qs + 4 * g) = h16x4{};
            *reinterpret_cast<h16x4*>(sDS + key_own * LDS_T + qs + 16 + 4 * g) = h16x4{};
          }
        }
        if (!any) continue;
        h16x8 pf[NKC], sf[NKC];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int q0 = qs + 16 * tt;
          f32x4 sc[NKC], dp[NKC];
#pragma unroll
          for (int j = 0; j < NKC; ++j) { sc[j] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[j] = sc[j]; }
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) {
            const h16x8 qf = frag_rows<HD>(sQ, q0, kk * 32, lane);
            const h16x8 df = frag_rows<HD>(sDO, q0, kk * 32, lane);
#pragma unroll
            for (int j = 0; j < NKC; ++j) {
              if (!act[j]) continue;
              sc[j] = mfma(qf, frag_rows<HD>(sK, 16 * w + 128 * j, kk * 32, lane), sc[j]);
              dp[j] = mfma(df, vf[j][kk], dp[j]);
            }
          }
          const f32x4 Lv = *reinterpret_cast<const f32x4*>(L + q0 + 4 * g);
          const f32x4 Dv = *reinterpret_cast<const f32x4*>(Dr + q0 + 4 * g);
#pragma unroll
          for (int j = 0; j < NKC; ++j) {
            if (!act[j]) continue;
            const int kw0 = 16 * w + 128 * j, key_own = kw0 + (lane & 15);
            // a 16x16 (query, key) tile valid everywhere (rows < Tq, keys < klen, causal: every key
            // at or before every row) skips the per-element masks
            const bool full = qbase + q0 + 15 < Tq && kw0 + 15 < klen && (!P.causal || kw0 + 15 <= qbase + q0);
            // dropout keep flags, branch-free; one mixer per element on the fast path
            bool keep[4] = {true, true, true, true};
            if (P.thresh) {
              const uint64_t c0 = zctr + (uint32_t)((qbase + q0 + 4 * g) * P.Tk + key_own);
              if (hi_pairs) {
                // lanes l, l^1 hold keys 2m, 2m+1 whose counters form one hash pair on every row
                // (even row stride and base): each lane mixes two of the four rows' pairs and the
                // lanes swap results (DPP quad_perm [1,0,3,2]) -- one mixer per two elements,
                // bit-identical to mms_keep_hi
                const bool odd = (lane & 1) != 0;
                const uint32_t p0 = (uint32_t)(c0 >> 1), st = (uint32_t)P.Tk >> 1;
                const uint32_t ha = mms_mix32((p0 + (odd ? 2 * st : 0u)) ^ hi_mix);
                const uint32_t hb = mms_mix32((p0 + (odd ? 3 * st : st)) ^ hi_mix);
                const uint32_t pa = (uint32_t)__builtin_amdgcn_mov_dpp((int)ha, 0xB1, 0xF, 0xF, false);
                const uint32_t pb = (uint32_t)__builtin_amdgcn_mov_dpp((int)hb, 0xB1, 0xF, 0xF, false);
                const uint32_t h4[4] = {odd ? pa : ha, odd ? pb : hb, odd ? ha : pa, odd ? hb : pb};
#pragma unroll
                for (int r = 0; r < 4; ++r) keep[r] = (odd ? h4[r] >> 16 : h4[r] & 0xffffu) >= P.thresh;
              } else if (hi_fast) {
#pragma unroll
                for (int r = 0; r < 4; ++r) keep[r] = mms_keep_hi(hi_mix, c0 + (uint32_t)(r * P.Tk), P.thresh);
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) keep[r] = mms_keep(P.seed, c0 + (uint32_t)(r * P.Tk), P.thresh);
              }
            }
            f32x4 pt, dst;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int q = qbase + q0 + 4 * g + r;
              const bool ok = full || (q < Tq && key_own < klen && (!P.causal || key_own <= q));
              const float e = __builtin_amdgcn_exp2f(fmaf(sc[j][r], c2, -Lv[r]));
              const float pr = ok ? e : 0.f;
              const float mk = keep[r] ? dscale : 0.f;
              pt[r] = pr * mk;
              dst[r] = pr * fmaf(dp[j][r], mk, -Dv[r]);
            }
            const h16x4 dh = h16x4{(h16)dst[0], (h16)dst[1], (h16)dst[2], (h16)dst[3]};
            *reinterpret_cast<h16x4*>(sDS + key_own * LDS_T + q0 + 4 * g) = dh;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              pf[j][4 * tt + r] = (h16)pt[r];
              sf[j][4 * tt + r] = dh[r];
            }
          }
        }
#pragma unroll
        for (int i = 0; i < NDT; ++i) {
          const h16x8 td = frag_tr<HD>(sDO, qs, 16 * i, lane);
          const h16x8 tq = frag_tr<HD>(sQ, qs, 16 * i, lane);
#pragma unroll
          for (int j = 0; j < NKC; ++j) {
            if (!act[j]) continue;
            dv[j][i] = mfma(td, pf[j], dv[j][i]);
            dk[j][i] = mfma(tq, sf[j], dk[j][i]);
          }
        }
      }
      if constexpr (LAST) {
        // dK, dV of the wave's own keys (keys in [klen, Tk) are written as zeros); then the next
        // head's K / V start loading behind phase 3.  Lane (key, g) holds d = 16i + 4g .. +3 of its
        // key row: with 16-B rows the lanes g and g ^ 1 (lane ^ 16, same key) swap halves so that
        // each stores 8 consecutive d (even g for even i, odd g for odd i) — half the store
        // instructions of the 8-B form, whose issue queue otherwise stalls phase 3's dQ stores.
        if (P.kv16) {
          typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
          const bool godd = (g & 1) != 0;
#pragma unroll
          for (int j = 0; j < NKC; ++j) {
            const int key_own = 16 * w + 128 * j + (lane & 15);
            h16* DK = P.dk + b * P.sdkb + h * HD + (long)key_own * P.lddk;
            h16* DV = P.dv + b * P.sdvb + h * HD + (long)key_own * P.lddv;
            const int gb = 4 * (g & 2);   // first d of the lane pair's 8-column group
#pragma unroll
            for (int i = 0; i < NDT; ++i) {
              const f32x4 a = dk[j][i] * P.scale, c = dv[j][i];
              const h16x4 ah = h16x4{(h16)a[0], (h16)a[1], (h16)a[2], (h16)a[3]};
              const h16x4 ch = h16x4{(h16)c[0], (h16)c[1], (h16)c[2], (h16)c[3]};
              typedef unsigned int u32x2_ __attribute__((ext_vector_type(2)));
              const u32x2_ au = __builtin_bit_cast(u32x2_, ah), cu = __builtin_bit_cast(u32x2_, ch);
              const u32x2_ ap = {(unsigned)__shfl_xor((int)au[0], 16, 64), (unsigned)__shfl_xor((int)au[1], 16, 64)};
              const u32x2_ cp = {(unsigned)__shfl_xor((int)cu[0], 16, 64), (unsigned)__shfl_xor((int)cu[1], 16, 64)};
              if (key_own < P.Tk && godd == ((i & 1) != 0)) {
                const u32x4_ ka = godd ? u32x4_{ap[0], ap[1], au[0], au[1]} : u32x4_{au[0], au[1], ap[0], ap[1]};
                const u32x4_ va = godd ? u32x4_{cp[0], cp[1], cu[0], cu[1]} : u32x4_{cu[0], cu[1], cp[0], cp[1]};
                *reinterpret_cast<u32x4_*>(DK + 16 * i + gb) = ka;
                *reinterpret_cast<u32x4_*>(DV + 16 * i + gb) = va;
              }
            }
          }
        } else {
#pragma unroll
        for (int j = 0; j < NKC; ++j) {
          const int key_own = 16 * w + 128 * j + (lane & 15);
          if (key_own < P.Tk) {
            h16* DK = P.dk + b * P.sdkb + h * HD + (long)key_own * P.lddk;
            h16* DV = P.dv + b * P.sdvb + h * HD + (long)key_own * P.lddv;
#pragma unroll
            for (int i = 0; i < NDT; ++i) {
              const f32x4 a = dk[j][i] * P.scale, c = dv[j][i];
              *reinterpret_cast<h16x4*>(DK + 16 * i + 4 * g) = h16x4{(h16)a[0], (h16)a[1], (h16)a[2], (h16)a[3]};
              *reinterpret_cast<h16x4*>(DV + 16 * i + 4 * g) = h16x4{(h16)c[0], (h16)c[1], (h16)c[2], (h16)c[3]};
            }
          }
        }
        }
        load_kv(znext < Z ? znext : z, znext < Z);
      }
      PH_STAMP(4 + 5 * gc);
      __syncthreads();
      PH_STAMP(5 + 5 * gc);
      // ---- phase 3: query tile w % NQT, d tiles (w / NQT)*NDW ..: dQ^T[d][q] = K^T[d][keys] dS^T[keys][q]
      {
        const int q0 = 16 * (w % NQT), qa0 = qbase + q0, d0 = (w / NQT) * NDW, q_own = qa0 + (lane & 15);
        if (qa0 < Tq) {
          const int kend = P.causal ? min(klen, qa0 + 16) : klen;
          f32x4 dq[NDW];
#pragma unroll
          for (int i = 0; i < NDW; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int kc = 0; kc < kend; kc += 32) {
            const h16x8 sf = frag_tr_ld<LDS_T>(sDS, kc, q0, lane);
#pragma unroll
            for (int i = 0; i < NDW; ++i) dq[i] = mfma(frag_tr<HD>(sK, kc, 16 * (d0 + i), lane), sf, dq[i]);
          }
          if (q_own < Tq) {
            h16* DQ = P.dq + b * P.sdqb + h * HD + (long)q_own * P.lddq;
#pragma unroll
            for (int i = 0; i < NDW; ++i) {
              const f32x4 a = dq[i] * P.scale;
              *reinterpret_cast<h16x4*>(DQ + 16 * (d0 + i) + 4 * g) = h16x4{(h16)a[0], (h16)a[1], (h16)a[2], (h16)a[3]};
            }
          }
        }
      }
      ++gc;
    };
    for (int ch = 0; ch + 1 < nch; ++ch) chunk(ch, std::false_type{});
    chunk(nch - 1, std::true_type{});
  }
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0)
      n = c;
    else
      n = 256;
  }
  return n;
}

template <typename F>
int pick_hd(int hd, F&& f) {
  switch (hd) {
    case 64: return f(std::integral_constant<int, 64>{});
    case 96: return f(std::integral_constant<int, 96>{});
    case 128: return f(std::integral_constant<int, 128>{});
    default: mms::set_error("flash attention: head_dim %d not supported (64/96/128)", hd); return 1;
  }
}

int check_common(const mms2ut_attn_args* a) {
  MMS_REQUIRE(a && a->q && a->k && a->v && a->o, "attention: null pointers");
  MMS_REQUIRE(a->B > 0 && a->H > 0 && a->Tq > 0 && a->Tk > 0, "attention: bad sizes");
  MMS_REQUIRE(a->ldq % 8 == 0 && a->ldk % 8 == 0 && a->ldv % 8 == 0 && a->ldo % 4 == 0,
              "attention: row strides must be multiples of 8 (q/k/v) and 4 (o)");
  MMS_REQUIRE(a->p < 1.f, "attention: dropout p must be < 1");
  return 0;
}

AttnP make_params(const mms2ut_attn_args* a) {
  AttnP P{};
  P.q = a->q; P.k = a->k; P.v = a->v; P.o = a->o;
  P.ldq = a->ldq; P.ldk = a->ldk; P.ldv = a->ldv; P.ldo = a->ldo;
  P.sqb = a->sqb ? a->sqb : (long)a->Tq * a->ldq;
  P.skb = a->skb ? a->skb : (long)a->Tk * a->ldk;
  P.svb = a->svb ? a->svb : (long)a->Tk * a->ldv;
  P.sob = a->sob ? a->sob : (long)a->Tq * a->ldo;
  P.H = a->H; P.Tq = a->Tq; P.Tk = a->Tk;
  P.key_len = a->key_len; P.causal = a->causal; P.scale = a->scale;
  P.p = a->p; P.thresh = mms_drop_thresh(a->p); P.seed = a->seed; P.offset = a->offset;
  P.lse = a->lse;
  return P;
}

}  // namespace

extern "C" int mms2ut_mha_varlen_fwd(const mms2ut_attn_args* a, hipStream_t s) {
  if (check_common(a)) return 1;
  MMS_REQUIRE(a->lse != nullptr, "attention fwd: lse buffer required");
  AttnP P = make_params(a);
  // each wave owns 16 query rows: 8 waves (128 rows) for Tq <= 128, else 16 waves (256 rows), so
  // that for every length up to 256 each (b, h) streams its K/V exactly once
  const int nw = a->Tq > 16 * ATTN_NW ? 2 * ATTN_NW : ATTN_NW;
  dim3 grid((a->Tq + 16 * nw - 1) / (16 * nw), a->B * a->H);
  return pick_hd(a->hd, [&](auto HDc) {
    constexpr int HD = decltype(HDc)::value;
    const bool short_k = a->Tk <= 2 * KB && P.ldk < (1L << 24) && P.ldv < (1L << 24);
    if (nw == ATTN_NW) {
      if (short_k) hipLaunchKernelGGL((attn_fwd_kernel<HD, ATTN_NW, true>), grid, dim3(64 * ATTN_NW), 0, s, P);
      else hipLaunchKernelGGL((attn_fwd_kernel<HD, ATTN_NW>), grid, dim3(64 * ATTN_NW), 0, s, P);
    } else {
      if (short_k) hipLaunchKernelGGL((attn_fwd_kernel<HD, 2 * ATTN_NW, true>), grid, dim3(128 * ATTN_NW), 0, s, P);
      else hipLaunchKernelGGL((attn_fwd_kernel<HD, 2 * ATTN_NW>), grid, dim3(128 * ATTN_NW), 0, s, P);
    }
    return mms::check_launch("mha_varlen_fwd");
  });
}

extern "C" int mms2ut_mha_varlen_bwd(const mms2ut_attn_args* a, const mms2ut_half* dout, int64_t lddo,
                                     int64_t sdob, float* Dd, mms2ut_half* dq, int64_t lddq, int64_t sdqb,
                                     mms2ut_half* dk, int64_t lddk, int64_t sdkb, mms2ut_half* dv,
                                     int64_t lddv, int64_t sdvb, hipStream_t s) {
  if (check_common(a)) return 1;
  MMS_REQUIRE(a->lse && dout && Dd && dq && dk && dv, "attention bwd: null buffers");
  MMS_REQUIRE(lddo % 8 == 0 && lddq % 4 == 0 && lddk % 4 == 0 && lddv % 4 == 0, "attention bwd: bad strides");
  AttnP P = make_params(a);
  P.dout = dout; P.lddo = lddo; P.sdob = sdob ? sdob : (long)a->Tq * lddo;
  P.Dd = Dd;
  P.dq = dq; P.lddq = lddq; P.sdqb = sdqb ? sdqb : (long)a->Tq * lddq;
  P.dk = dk; P.lddk = lddk; P.sdkb = sdkb ? sdkb : (long)a->Tk * lddk;
  P.dv = dv; P.lddv = lddv; P.sdvb = sdvb ? sdvb : (long)a->Tk * lddv;
  {
    P.kv16 = P.lddk % 8 == 0 && P.lddv % 8 == 0 && P.sdkb % 8 == 0 && P.sdvb % 8 == 0 &&
             (a->hd % 16) == 0 && ((uintptr_t)P.dk & 15) == 0 && ((uintptr_t)P.dv & 15) == 0;
  }
  const int Z = a->B * a->H;
  const bool fused_ok = a->Tk <= 256 && a->hd <= 96 &&
                        P.ldo % 8 == 0 && P.sob % 8 == 0 && ((uintptr_t)P.o & 15) == 0 &&
                        P.lddo % 8 == 0 && P.sdob % 8 == 0 && ((uintptr_t)P.dout & 15) == 0;
  if (fused_ok) {
    return pick_hd(a->hd, [&](auto HDc) {
      constexpr int HD = decltype(HDc)::value;
      if constexpr (HD <= 96) {
        // persistent grid: one block per CU (the kernel's LDS allows no second), each looping
        // over heads so that the next head's loads overlap the current head's MFMA phases
        const int grid = std::min(Z, num_cus());
        if (a->Tk <= 128)
          hipLaunchKernelGGL((attn_bwd_fused_kernel<HD, 1>), dim3(grid), dim3(512), 0, s, P, Z);
        else
          hipLaunchKernelGGL((attn_bwd_fused_kernel<HD, 2>), dim3(grid), dim3(512), 0, s, P, Z);
        return mms::check_launch("mha_varlen_bwd_fused");
      } else {
        mms::set_error("unreachable");
        return 1;
      }
    });
  }
  return pick_hd(a->hd, [&](auto HDc) {
    constexpr int HD = decltype(HDc)::value;
    const bool rows_ok = a->H <= 64 && 64 % a->H == 0 && (HD / 4) % (64 / a->H) == 0 &&
                         P.ldo % 4 == 0 && P.lddo % 4 == 0 && P.sob % 4 == 0 && P.sdob % 4 == 0 &&
                         ((uintptr_t)P.o & 7) == 0 && ((uintptr_t)P.dout & 7) == 0;
    if (rows_ok) {
      const long nrows = (long)a->B * a->Tq;
      hipLaunchKernelGGL((attn_bwd_prep_rows_kernel<HD>), dim3((nrows + 3) / 4), dim3(256), 0, s, P, nrows);
    } else {
      hipLaunchKernelGGL((attn_bwd_prep_kernel<HD>), dim3(((long)Z * a->Tq + 3) / 4), dim3(256), 0, s, P, Z);
    }
    if (int rc = mms::check_launch("mha_varlen_bwd_prep")) return rc;
    constexpr int OWN = 16 * ATTN_NW;
    hipLaunchKernelGGL((attn_bwd_kv_kernel<HD, ATTN_NW>), dim3((a->Tk + OWN - 1) / OWN, Z), dim3(64 * ATTN_NW), 0, s, P);
    if (int rc = mms::check_launch("mha_varlen_bwd_kv")) return rc;
    hipLaunchKernelGGL((attn_bwd_q_kernel<HD, ATTN_NW>), dim3((a->Tq + OWN - 1) / OWN, Z), dim3(64 * ATTN_NW), 0, s, P);
    return mms::check_launch("mha_varlen_bwd_q");
  });
}

namespace mms {
int bind_step_seed_attention(const uint64_t* d) { return mms_bind_step_seed_tu(d); }
}  // namespace mms

#ifdef MMS_ATTN_PHASES
extern "C" int mms2ut_diag_attn_phases(unsigned long long* host, int n, int clear) {
  if (clear) {
    static unsigned long long zero[64 * 64] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_attn_ph), zero, sizeof(zero)) != hipSuccess;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_ph), sizeof(unsigned long long) * (n < 4096 ? n : 4096)) != hipSuccess;
}
#endif
