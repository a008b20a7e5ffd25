// Beam-search decoding support (fairseq-generate --beam 10 over the unit decoder).
//   * log_softmax_step: fairseq SequenceGenerator._generate's per-step normalisation of the
//     decoder output (model.get_normalized_probs(log_probs=True) = log_softmax(logits.float()))
//     fused with its masking: NaN -> -inf, <pad> -> -inf, and at step >= max_len every token but
//     </s> -> -inf, or before min_len </s> -> -inf.  One wave per hypothesis row.
//   * kv_cache_gather: reorder_incremental_state — every decoder layer's self-attention K|V cache
//     rows [0, rows) of hypothesis idx[n] (of the Nsrc previous slots) copied to slot n of the N
//     new ones (the batch shrinks as sentences finish), 16-B vectors, grid-stride.
#include <algorithm>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

__global__ void __launch_bounds__(256) log_softmax_step_kernel(const h16* __restrict__ z, long ld, long rows,
                                                               int V, int pad, int eos, int mode,
                                                               float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const h16* zr = z + row * ld;
  float mx = -INFINITY;
  for (int j = lane; j < V; j += 64) {
    const float v = (float)zr[j];
    if (v == v) mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  float se = 0.f;
  for (int j = lane; j < V; j += 64) {
    const float v = (float)zr[j];
    if (v == v && v != -INFINITY) se += expf(v - mx);
  }
  se = wave_sum(se);
  const float lse = mx + logf(se);
  float* o = out + row * (long)V;
  for (int j = lane; j < V; j += 64) {
    const float v = (float)zr[j];
    float r = (v == v) ? v - lse : -INFINITY;
    if (j == pad) r = -INFINITY;
    if (mode == 1 && j != eos) r = -INFINITY;
    if (mode == 2 && j == eos) r = -INFINITY;
    o[j] = r;
  }
}

__global__ void __launch_bounds__(256) kv_cache_gather_kernel(const h16* __restrict__ src, h16* __restrict__ dst,
                                                              const int64_t* __restrict__ idx, int L, int Nsrc,
                                                              int N, int maxT, int rows, int width) {
  const int vw = width / 8;                       // 16-B vectors per cache row
  const long per_slot = (long)rows * vw;
  const long total = (long)L * N * per_slot;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long ln = i / per_slot, r = i % per_slot;
    const int l = (int)(ln / N), n = (int)(ln % N);
    const long sbase = ((long)l * Nsrc + idx[n]) * maxT * width;
    const long dbase = ((long)l * N + n) * maxT * width;
    reinterpret_cast<s16x8*>(dst + dbase)[r] = reinterpret_cast<const s16x8*>(src + sbase)[r];
  }
}

// One decoder step of self-attention over the cache, addressed through a slot table (so a beam
// reorder moves N*T int32 indices instead of every layer's K/V rows): key/value row t of
// hypothesis n is row t of cache slot slot[n][t].  One 256-thread block per (hypothesis, head):
// phase 1 — threads over keys, q.k by packed fp16 dot products (q in registers), scores and row
// offsets to LDS, block max / sum; phase 2 — HD/8 threads per V row (16-B loads), 256/(HD/8) rows
// in flight, fp32 partials reduced across row groups through LDS; output fp16.  Reads
// T*hd*2*2 B per (hypothesis, head): HBM/latency-bound.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
constexpr int DEC_THREADS = 256;

template <int HD>
__global__ void __launch_bounds__(DEC_THREADS) decode_attn_kernel(const h16* __restrict__ q, long ldq,
                                                                  h16* __restrict__ cache, int* __restrict__ slot,
                                                                  int H, int maxT, const int* __restrict__ step_ptr,
                                                                  const h16* __restrict__ kv_new, long ld_new,
                                                                  long width, h16* __restrict__ out, long ldo,
                                                                  float scale) {
  constexpr int VL = HD / 8;                  // threads per V row (16-B vectors)
  constexpr int G = DEC_THREADS / VL;         // V rows in flight
  extern __shared__ float s_dyn[];
  float* s_p = s_dyn;                                           // [maxT] scores -> probabilities
  long* s_off = reinterpret_cast<long*>(s_dyn + ((maxT + 1) & ~1));  // [maxT] element offsets of the rows
  __shared__ float s_part[G][HD];
  __shared__ float s_red[DEC_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = blockIdx.x / H, h = blockIdx.x % H;
  // T = step + 1 read on the device (graph-replayable); row T-1 is this step's K|V, taken from the
  // projection's staging rows and stored into row T-1 of slot n for the steps that follow
  const int T = min(*step_ptr + 1, maxT);
  const h16* kvn = kv_new + (long)n * ld_new;
  if (tid < 2 * VL) {
    const long col = (tid < VL ? 0 : width / 2) + h * HD + (tid % VL) * 8;
    *reinterpret_cast<s16x8*>(cache + ((long)n * maxT + (T - 1)) * width + col) =
        *reinterpret_cast<const s16x8*>(kvn + col);
  }
  if (h == 0 && tid == 0) slot[(long)n * maxT + T - 1] = n;
  s16x8 qv[VL];
  const h16* qr = q + (long)n * ldq + h * HD;
#pragma unroll
  for (int i = 0; i < VL; ++i) qv[i] = reinterpret_cast<const s16x8*>(qr)[i];
  const int* sl = slot + (long)n * maxT;   // entry T-1 is n (written above, not read back)
  float mx = -INFINITY;
  for (int t = tid; t < T; t += DEC_THREADS) {
    const long off = ((long)sl[t] * maxT + t) * width + h * HD;
    const h16* kr = t == T - 1 ? kvn + h * HD : cache + off;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const h16x8 kk = __builtin_bit_cast(h16x8, reinterpret_cast<const s16x8*>(kr)[i]);
      const h16x8 qq = __builtin_bit_cast(h16x8, qv[i]);
#pragma unroll
      for (int e = 0; e < 8; e += 2)
        acc = __builtin_amdgcn_fdot2(h16x2{qq[e], qq[e + 1]}, h16x2{kk[e], kk[e + 1]}, acc, false);
    }
    acc *= scale;
    s_p[t] = acc;
    s_off[t] = off;
    mx = fmaxf(mx, acc);
  }
  mx = wave_max(mx);
  if (lane == 0) s_red[w] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int t = tid; t < T; t += DEC_THREADS) {
    const float e = __expf(s_p[t] - mx);
    s_p[t] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) s_red[w] = sum;
  __syncthreads();
  const float inv = 1.f / ((s_red[0] + s_red[1]) + (s_red[2] + s_red[3]));
  const int g = tid / VL, c = tid % VL;
  if (g < G) {
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const long vcol = width / 2 + c * 8;
#pragma unroll 4
    for (int t = g; t < T; t += G) {
      const h16* vr = t == T - 1 ? kvn + h * HD + vcol : cache + s_off[t] + vcol;
      const h16x8 v = __builtin_bit_cast(h16x8, *reinterpret_cast<const s16x8*>(vr));
      const float pt = s_p[t];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pt * (float)v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s_part[g][c * 8 + e] = o[e];
  }
  __syncthreads();
  if (tid < HD) {
    float a = 0.f;
#pragma unroll
    for (int gg = 0; gg < G; ++gg) a += s_part[gg][tid];
    out[(long)n * ldo + h * HD + tid] = (h16)(a * inv);
  }
}

// Split-K epilogue for the decoder step's small-M GEMMs (M = hypotheses, ~100-300 rows: one or two
// tile rows, so K = 768 / 3072 runs as a long serial k-loop on a dozen blocks): the GEMM writes
// `nsplit` fp32 slabs, this sums them and applies the layer's epilogue — + bias, ReLU, + residual
// — to fp16 (the same arithmetic as the fused GEMM epilogue, summed in fp32).
__global__ void __launch_bounds__(256) splitk_epilogue_kernel(const float* __restrict__ slabs, int nsplit, long slab,
                                                              int M, int N, const h16* __restrict__ bias,
                                                              const h16* __restrict__ aux, long ldaux, int relu,
                                                              h16* __restrict__ out, long ldo) {
  const long nv = (long)M * N / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long)gridDim.x * blockDim.x) {
    const long e = 4 * i;
    const int r = (int)(e / N), c = (int)(e % N);
    f32x4 a = *reinterpret_cast<const f32x4*>(slabs + e);
    for (int k = 1; k < nsplit; ++k) a += *reinterpret_cast<const f32x4*>(slabs + k * slab + e);
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = a[j];
      if (bias) v += (float)bias[c + j];
      if (relu) v = fmaxf(v, 0.f);
      o[j] = v;
    }
    if (aux) {
      const h16x4 x = *reinterpret_cast<const h16x4*>(aux + (long)r * ldaux + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (float)(h16)o[j] + (float)x[j];
    }
    h16x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = (h16)o[j];
    *reinterpret_cast<h16x4*>(out + (long)r * ldo + c) = y;
  }
}

// fairseq TransformerDecoder embedding for one incremental step: x[n] = scale * E[tok[n]] +
// pos[pad + 1 + step] (SinusoidalPositionalEmbedding with incremental_state), step read on the
// device so the decoder step can be replayed as a graph.  fp32 arithmetic, one fp16 rounding (as
// token_embed_fwd).  One wave per hypothesis row.
__global__ void __launch_bounds__(256) decode_embed_kernel(const int64_t* __restrict__ tok, const h16* __restrict__ E,
                                                           const h16* __restrict__ pos, const int* __restrict__ step_ptr,
                                                           int pad, h16* __restrict__ x, int N, int D, float scale) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const long prow = (long)(pad + 1 + *step_ptr) * D;
  const long erow = tok[n] * (long)D;
  for (int d0 = lane * 4; d0 < D; d0 += 256) {
    const h16x4 ev = *reinterpret_cast<const h16x4*>(E + erow + d0);
    const h16x4 pv = *reinterpret_cast<const h16x4*>(pos + prow + d0);
    h16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (h16)(scale * (float)ev[e] + (float)pv[e]);
    *reinterpret_cast<h16x4*>(x + (long)n * D + d0) = o;
  }
}

// The decoder step's residual projections (out_proj, encoder_attn.out_proj, fc2) are followed by a
// LayerNorm of their output: x = fp16(fp16(sum of slabs + bias) + residual), y = LN(x) — in one
// launch (one wave per hypothesis row, the row in registers).  Same arithmetic, summation order and
// roundings as splitk_epilogue_kernel followed by ln_fwd_kernel, so the fused step is bit-identical.
template <int CPL>
__global__ void __launch_bounds__(256) splitk_epilogue_ln_kernel(const float* __restrict__ slabs, int nsplit,
                                                                 long slab, int M, int N,
                                                                 const h16* __restrict__ bias,
                                                                 const h16* __restrict__ aux, long ldaux,
                                                                 h16* __restrict__ xout, long ldx,
                                                                 const h16* __restrict__ g, const h16* __restrict__ b,
                                                                 float eps, h16* __restrict__ y, long ldy) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = N >> 2;
  float v[CPL][4];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[c][e] = 0.f;
    if (ch < nch) {
      const long off = (long)row * N + ch * 4;
      f32x4 a = *reinterpret_cast<const f32x4*>(slabs + off);
      for (int k = 1; k < nsplit; ++k) a += *reinterpret_cast<const f32x4*>(slabs + k * slab + off);
      const h16x4 r = *reinterpret_cast<const h16x4*>(aux + (long)row * ldaux + ch * 4);
      h16x4 xo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = a[e];
        if (bias) t += (float)bias[ch * 4 + e];
        xo[e] = (h16)((float)(h16)t + (float)r[e]);
        v[c][e] = (float)xo[e];
        sum += v[c][e];
      }
      *reinterpret_cast<h16x4*>(xout + (long)row * ldx + ch * 4) = xo;
    }
  }
  const float mean = wave_sum(sum) / N;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c)
    if (lane + c * 64 < nch) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[c][e] - mean; ss += d * d; }
    }
  const float rstd = rsqrtf(wave_sum(ss) / N + eps);
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      const h16x4 gg = *reinterpret_cast<const h16x4*>(g + ch * 4), bb = *reinterpret_cast<const h16x4*>(b + ch * 4);
      h16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (h16)((v[c][e] - mean) * rstd * (float)gg[e] + (float)bb[e]);
      *reinterpret_cast<h16x4*>(y + (long)row * ldy + ch * 4) = o;
    }
  }
}

// BeamSearch.step's candidate selection for one step: per sentence b, the top k of
// lprobs[b, j, v] + scores[b*beam + j] over (j, v) (only j = 0 at step 0, when every beam holds
// the same prefix), in descending score order, ties to the lower flat index j*V + v.  Keys are
// 64-bit (order-preserving score bits | inverted index), so a max is a unique candidate.  Replaces
// torch.topk over [bsz, beam*V].
MMS_DEV uint64_t beam_key(float v, uint32_t idx) {
  uint32_t u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((uint64_t)u << 32) | (uint64_t)(0xFFFFFFFFu - idx);
}

MMS_DEV uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    const uint64_t w = ((uint64_t)hi << 32) | lo;
    v = w > v ? w : v;
  }
  return v;
}

// Two passes, spreading a sentence over BT_PARTS waves (a one-block-per-sentence form keeps a
// sentence on one CU and measured slower): pass 1 — each wave takes a contiguous share of the sentence's
// candidates, keeps a per-lane register top-k and pops its own top k by k wave-max rounds into
// part[b][p][k] (key 0 = empty); pass 2 — one wave per sentence merges the BT_PARTS*k keys the same
// way and decodes them.  The keys are unique (flat index in the low word), so the result equals a
// global sort exactly.
constexpr int BT_PARTS = 32;

template <int KK>
MMS_DEV void lane_insert(uint64_t (&top)[KK], uint64_t x) {
  if (x > top[KK - 1]) {
#pragma unroll
    for (int t = 0; t < KK; ++t) {
      const uint64_t hi = x > top[t] ? x : top[t], lo = x > top[t] ? top[t] : x;
      top[t] = hi;
      x = lo;
    }
  }
}

template <int KK>
MMS_DEV uint64_t wave_pop(uint64_t (&top)[KK]) {
  const uint64_t m = wave_max_u64(top[0]);
  if (top[0] == m && m != 0) {
#pragma unroll
    for (int t = 0; t < KK - 1; ++t) top[t] = top[t + 1];
    top[KK - 1] = 0;
  }
  return m;
}

template <int KK>
__global__ void __launch_bounds__(256) beam_topk_part_kernel(const float* __restrict__ lprobs,
                                                             const float* __restrict__ prev, long ld_prev, int beam,
                                                             int V, int jmax, int k, int bsz,
                                                             uint64_t* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= bsz * BT_PARTS) return;
  const int b = gw / BT_PARTS, p = gw % BT_PARTS;
  const int n = jmax * V, chunk = (n + BT_PARTS - 1) / BT_PARTS;
  const int i0 = p * chunk, i1 = min(n, i0 + chunk);
  uint64_t top[KK];
#pragma unroll
  for (int i = 0; i < KK; ++i) top[i] = 0;
  for (int i = i0 + lane; i < i1; i += 64) {
    const int j = i / V, v = i - j * V;
    float sc = lprobs[((long)b * beam + j) * V + v];
    if (prev) sc += prev[((long)b * beam + j) * ld_prev];
    lane_insert<KK>(top, beam_key(sc, (uint32_t)i));
  }
  for (int r = 0; r < k; ++r) {
    const uint64_t m = wave_pop<KK>(top);
    if (lane == 0) part[((long)b * BT_PARTS + p) * k + r] = m;
  }
}

template <int KK>
__global__ void __launch_bounds__(64) beam_topk_merge_kernel(const uint64_t* __restrict__ part, int k, int V,
                                                             float* __restrict__ out_score,
                                                             int64_t* __restrict__ out_tok,
                                                             int64_t* __restrict__ out_beam) {
  const int lane = threadIdx.x, b = blockIdx.x;
  uint64_t top[KK];
#pragma unroll
  for (int i = 0; i < KK; ++i) top[i] = 0;
  const uint64_t* pb = part + (long)b * BT_PARTS * k;
  for (int i = lane; i < BT_PARTS * k; i += 64) lane_insert<KK>(top, pb[i]);
  for (int r = 0; r < k; ++r) {
    const uint64_t best = wave_pop<KK>(top);
    if (lane == 0) {
      const uint32_t idx = 0xFFFFFFFFu - (uint32_t)best;
      uint32_t u = (uint32_t)(best >> 32);
      u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
      out_score[(long)b * k + r] = __uint_as_float(u);
      out_tok[(long)b * k + r] = idx % V;
      out_beam[(long)b * k + r] = idx / V;
    }
  }
}

}  // namespace

extern "C" int mms2ut_log_softmax_step(const h16* logits, int64_t ld, int64_t rows, int V, int pad_idx,
                                       int eos_idx, int mode, float* lprobs, hipStream_t s) {
  MMS_REQUIRE(ld >= V && V > 0, "log_softmax_step: ld must be >= V > 0");
  MMS_REQUIRE(mode >= 0 && mode <= 2, "log_softmax_step: mode must be 0, 1 or 2");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(log_softmax_step_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, logits, (long)ld,
                     (long)rows, V, pad_idx, eos_idx, mode, lprobs);
  return mms::check_launch("log_softmax_step");
}

extern "C" int mms2ut_kv_cache_gather(const h16* src, h16* dst, const int64_t* idx, int L, int Nsrc, int N,
                                      int maxT, int rows, int width, hipStream_t s) {
  MMS_REQUIRE(width % 8 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0,
              "kv_cache_gather: width % 8 and 16-B alignment required");
  MMS_REQUIRE(rows >= 0 && rows <= maxT, "kv_cache_gather: rows must be in [0, maxT]");
  const long total = (long)L * N * rows * (width / 8);
  if (total == 0) return 0;
  const int nb = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(kv_cache_gather_kernel, dim3(nb), dim3(256), 0, s, src, dst, idx, L, Nsrc, N, maxT, rows,
                     width);
  return mms::check_launch("kv_cache_gather");
}

extern "C" int mms2ut_decode_self_attn(const h16* q, int64_t ldq, h16* cache, int32_t* slot, int N, int H,
                                       int hd, int maxT, const int32_t* step, const h16* kv_new, int64_t ld_new,
                                       int64_t width, h16* out, int64_t ldo, float scale, hipStream_t s) {
  MMS_REQUIRE(width == 2L * H * hd && ldq % 8 == 0 && width % 8 == 0 && ld_new % 8 == 0,
              "decode_self_attn: width must be 2*H*hd, ldq / width / ld_new multiples of 8");
  const size_t lds = (size_t)((maxT + 1) & ~1) * 4 + (size_t)maxT * 8;
  MMS_REQUIRE(lds <= 64 * 1024, "decode_self_attn: maxT too long for the LDS score rows (<= 5400)");
  if (N == 0) return 0;
  const dim3 grid(N * H);
  switch (hd) {
#define CASE(HD) case HD: hipLaunchKernelGGL(decode_attn_kernel<HD>, grid, dim3(DEC_THREADS), lds, s, q, (long)ldq, \
                                             cache, slot, H, maxT, step, kv_new, (long)ld_new, (long)width, out, \
                                             (long)ldo, scale); break;
    CASE(64) CASE(96) CASE(128)
#undef CASE
    default: mms::set_error("decode_self_attn: head dim must be 64, 96 or 128"); return 1;
  }
  return mms::check_launch("decode_self_attn");
}

extern "C" int mms2ut_decode_embed(const int64_t* tok, const h16* E, const h16* pos, const int32_t* step, int pad_idx,
                                   h16* x, int N, int D, float scale, hipStream_t s) {
  MMS_REQUIRE(D % 4 == 0, "decode_embed: D must be a multiple of 4");
  if (N == 0) return 0;
  hipLaunchKernelGGL(decode_embed_kernel, dim3((N + 3) / 4), dim3(256), 0, s, tok, E, pos, step, pad_idx, x, N, D,
                     scale);
  return mms::check_launch("decode_embed");
}

extern "C" int mms2ut_splitk_epilogue_f16(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                                          const h16* bias, const h16* aux, int64_t ldaux, int relu, h16* out,
                                          int64_t ldo, hipStream_t s) {
  MMS_REQUIRE(cols % 4 == 0 && ldo % 4 == 0 && (!aux || ldaux % 4 == 0) && slab % 4 == 0,
              "splitk_epilogue: cols / strides must be multiples of 4");
  MMS_REQUIRE(nsplit >= 1, "splitk_epilogue: nsplit >= 1");
  const long nv = (long)rows * cols / 4;
  if (nv == 0) return 0;
  const int nb = (int)std::min<long>((nv + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(nb), dim3(256), 0, s, slabs, nsplit, (long)slab, rows, cols,
                     bias, aux, (long)ldaux, relu, out, (long)ldo);
  return mms::check_launch("splitk_epilogue");
}

extern "C" int mms2ut_splitk_epilogue_ln_f16(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                                             const h16* bias, const h16* aux, int64_t ldaux, h16* xout, int64_t ldx,
                                             const h16* gamma, const h16* beta, float eps, h16* y, int64_t ldy,
                                             hipStream_t s) {
  MMS_REQUIRE(cols % 4 == 0 && cols <= 1024 && ldaux % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && slab % 4 == 0,
              "splitk_epilogue_ln: cols <= 1024 and strides must be multiples of 4");
  MMS_REQUIRE(aux != nullptr && gamma != nullptr && beta != nullptr, "splitk_epilogue_ln: aux, gamma, beta required");
  if (rows == 0) return 0;
  const int cpl = (cols / 4 + 63) / 64;
  const dim3 grid((rows + 3) / 4);
  switch (cpl) {
#define CASE(C) case C: hipLaunchKernelGGL(splitk_epilogue_ln_kernel<C>, grid, dim3(256), 0, s, slabs, nsplit, \
                                           (long)slab, rows, cols, bias, aux, (long)ldaux, xout, (long)ldx, gamma, \
                                           beta, eps, y, (long)ldy); break;
    CASE(1) CASE(2) CASE(3) CASE(4)
#undef CASE
  }
  return mms::check_launch("splitk_epilogue_ln");
}

extern "C" int mms2ut_beam_topk(const float* lprobs, const float* prev_scores, int64_t ld_prev, int bsz, int beam,
                                int V, int first_step, int k, float* out_score, int64_t* out_tok,
                                int64_t* out_beam, uint64_t* work, hipStream_t s) {
  const int jmax = first_step ? 1 : beam;
  MMS_REQUIRE(k >= 1 && k <= 32 && k < jmax * V, "beam_topk: need 1 <= k <= 32 and k < candidates");
  MMS_REQUIRE((long)beam * V < 0x7FFFFFFFL, "beam_topk: beam * V too large");
  if (bsz == 0) return 0;
  const float* prev = first_step ? nullptr : prev_scores;
  const int kk = k <= 8 ? 8 : k <= 16 ? 16 : k <= 24 ? 24 : 32;
  MMS_REQUIRE(work != nullptr, "beam_topk: work buffer (bsz * 32 * k uint64) required");
  const dim3 g1((bsz * BT_PARTS + 3) / 4);
  switch (kk) {
#define CASE(KK) case KK: \
    hipLaunchKernelGGL(beam_topk_part_kernel<KK>, g1, dim3(256), 0, s, lprobs, prev, (long)ld_prev, beam, V, jmax, \
                       k, bsz, work); \
    hipLaunchKernelGGL(beam_topk_merge_kernel<KK>, dim3(bsz), dim3(64), 0, s, work, k, V, out_score, out_tok, \
                       out_beam); break;
    CASE(8) CASE(16) CASE(24) CASE(32)
#undef CASE
  }
  return mms::check_launch("beam_topk");
}
