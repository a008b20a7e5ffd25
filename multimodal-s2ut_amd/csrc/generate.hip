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
