// Shared device/host helpers for libmms2ut_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 h16;
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define MMS_DEV __device__ __forceinline__

// ------------------------------------------------------------------------------------------
// error plumbing (host): every C-ABI entry returns 0 or a status; text in mms2ut_last_error()
// ------------------------------------------------------------------------------------------
namespace mms {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
}  // namespace mms

#define MMS_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      mms::set_error(__VA_ARGS__);        \
      return 1;                           \
    }                                     \
  } while (0)

// ------------------------------------------------------------------------------------------
// counter-based dropout RNG: keep(i) is a pure function of (seed, offset + i) so the backward
// pass regenerates the forward mask without storing it.  Same stream for every kernel.
// ------------------------------------------------------------------------------------------
// 32-bit integer mixer (lowbias32: two 32-bit multiplies) — cheap enough for GEMM epilogues.
MMS_DEV uint32_t mms_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// one 32-bit draw per PAIR of counters (ctr>>1); element ctr takes the low/high 16 bits.
// keep(ctr) <=> u16 >= thresh16 with thresh16 = round(p * 65536): P(drop) = p to 1.5e-5.
MMS_DEV uint32_t mms_hash(uint64_t seed, uint64_t ctr) {
  const uint64_t pair = ctr >> 1;
  const uint32_t s = (uint32_t)seed ^ mms_mix32((uint32_t)(seed >> 32) + 0x9e3779b9U);
  const uint32_t h = mms_mix32((uint32_t)pair ^ mms_mix32((uint32_t)(pair >> 32) ^ s));
  return (ctr & 1) ? (h >> 16) : (h & 0xffffU);
}
MMS_DEV bool mms_keep(uint64_t seed, uint64_t ctr, uint32_t thresh) {
  return mms_hash(seed, ctr) >= thresh;
}
// keep-flags of 4 consecutive counters ctr0..ctr0+3 (2 hashes when ctr0 is even)
MMS_DEV void mms_keep4(uint64_t seed, uint64_t ctr0, uint32_t thresh, bool (&k)[4]) {
  if ((ctr0 & 1) == 0) {
    const uint32_t s = (uint32_t)seed ^ mms_mix32((uint32_t)(seed >> 32) + 0x9e3779b9U);
    const uint64_t p0 = ctr0 >> 1;
    const uint32_t h0 = mms_mix32((uint32_t)p0 ^ mms_mix32((uint32_t)(p0 >> 32) ^ s));
    const uint64_t p1 = p0 + 1;
    const uint32_t h1 = mms_mix32((uint32_t)p1 ^ mms_mix32((uint32_t)(p1 >> 32) ^ s));
    k[0] = (h0 & 0xffffU) >= thresh;
    k[1] = (h0 >> 16) >= thresh;
    k[2] = (h1 & 0xffffU) >= thresh;
    k[3] = (h1 >> 16) >= thresh;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) k[e] = mms_keep(seed, ctr0 + e, thresh);
  }
}
// Fast path of mms_hash for a run of counters whose pair index (ctr >> 1) shares one high word:
// the seed / high-word half of the hash is a per-run constant mms_hi_mix(seed, ctr0); every
// element then costs one mixer instead of two.  Bit-identical to mms_keep on that run.
MMS_DEV uint32_t mms_hi_mix(uint64_t seed, uint64_t ctr0) {
  const uint32_t s = (uint32_t)seed ^ mms_mix32((uint32_t)(seed >> 32) + 0x9e3779b9U);
  return mms_mix32((uint32_t)((ctr0 >> 1) >> 32) ^ s);
}
MMS_DEV bool mms_same_hi(uint64_t ctr0, uint64_t ctr_last) { return ((ctr0 >> 1) >> 32) == ((ctr_last >> 1) >> 32); }
MMS_DEV bool mms_keep_hi(uint32_t hi_mix, uint64_t ctr, uint32_t thresh) {
  const uint32_t h = mms_mix32((uint32_t)(ctr >> 1) ^ hi_mix);
  return ((ctr & 1) ? (h >> 16) : (h & 0xffffU)) >= thresh;
}
MMS_DEV void mms_keep4_hi(uint32_t hi_mix, uint64_t ctr0, uint32_t thresh, bool (&k)[4]) {
  if ((ctr0 & 1) == 0) {
    const uint32_t p0 = (uint32_t)(ctr0 >> 1);
    const uint32_t h0 = mms_mix32(p0 ^ hi_mix), h1 = mms_mix32((p0 + 1) ^ hi_mix);
    k[0] = (h0 & 0xffffU) >= thresh;
    k[1] = (h0 >> 16) >= thresh;
    k[2] = (h1 & 0xffffU) >= thresh;
    k[3] = (h1 >> 16) >= thresh;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) k[e] = mms_keep_hi(hi_mix, ctr0 + e, thresh);
  }
}
// A dropout site's hash constant hoisted out of the per-element work: when every counter pair of the
// site [ctr0, ctr_last] shares one high word (always, unless the site straddles a 2^33 boundary)
// a keep flag costs one mixer per counter pair instead of two (bit-identical to mms_keep*).
struct MmsSite {
  bool hi;
  uint32_t mix;
};
MMS_DEV MmsSite mms_site(uint64_t seed, uint64_t ctr0, uint64_t ctr_last) {
  MmsSite s;
  s.hi = mms_same_hi(ctr0, ctr_last);
  s.mix = s.hi ? mms_hi_mix(seed, ctr0) : 0u;
  return s;
}
MMS_DEV void mms_keep4_site(const MmsSite& s, uint64_t seed, uint64_t ctr0, uint32_t thresh, bool (&k)[4]) {
  if (s.hi) mms_keep4_hi(s.mix, ctr0, thresh, k);
  else mms_keep4(seed, ctr0, thresh, k);
}
MMS_DEV bool mms_keep_site(const MmsSite& s, uint64_t seed, uint64_t ctr, uint32_t thresh) {
  return s.hi ? mms_keep_hi(s.mix, ctr, thresh) : mms_keep(seed, ctr, thresh);
}
// Step-seed indirection for HIP-graph replay.  A captured launch keeps the host seed it was
// captured with; the per-step variation comes from a device-resident 64-bit delta that every
// dropout kernel adds to its seed argument on entry (the step's first kernel advances it, see
// mms2ut_step_seed_advance).  Unbound (the eager default) => delta 0, masks unchanged.  One copy
// of the pointer per translation unit; mms2ut_bind_step_seed binds all of them.
static __device__ const uint64_t* mms_step_seed_delta = nullptr;
MMS_DEV uint64_t mms_step_seed(uint64_t s) {
  const uint64_t* d = mms_step_seed_delta;
  return d ? s + *d : s;
}
static inline int mms_bind_step_seed_tu(const uint64_t* d) {
  return hipMemcpyToSymbol(HIP_SYMBOL(mms_step_seed_delta), &d, sizeof(d)) == hipSuccess ? 0 : 1;
}
static inline uint32_t mms_drop_thresh(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 65536.0 + 0.5;
  if (t >= 65536.0) return 65536u;
  if (t < 1.0) t = 1.0;
  return (uint32_t)t;
}

// ------------------------------------------------------------------------------------------
// wave64 reductions without LDS.  __shfl_xor lowers to ds_bpermute_b32 on gfx950 — an LDS round
// trip (tens of cycles) per step, six of them in series for a wave sum, on the critical path of
// every LayerNorm row and softmax tile.  Here: DPP row rotates (8, 4, 2, 1) inside each 16-lane
// row, then gfx950's v_permlane16_swap / v_permlane32_swap across rows (plain VALU).  Every stage
// adds (or maxes) a value with its partner in the same order on both lanes, so all 64 lanes end
// with bit-identical results.  Call from wave-uniform control flow (all lanes active).
// ------------------------------------------------------------------------------------------
template <int CTRL>
MMS_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_ROR8 = 0x128, DPP_ROR4 = 0x124, DPP_ROR2 = 0x122, DPP_ROR1 = 0x121;
// the two values of lane pairs (l, l ^ 16) / (l, l ^ 32): .x = the lower row's, .y = the upper's
struct f32pair { float lo, hi; };
// The swap is written as inline asm: through the builtins, ROCm 7.2's compiler folds the two
// results of a swap whose results are combined in one expression into the first one
// (v_permlane16_swap v0, v1; v_add_f32 v0, v0, v0 — scripts/micro/permlane_probe.hip).  The
// s_nop covers the VALU-write -> permlane-read hazard the compiler would otherwise insert.
MMS_DEV f32pair xpair16(float v) {
  unsigned a = __builtin_bit_cast(unsigned, v), b = a;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return {__builtin_bit_cast(float, a), __builtin_bit_cast(float, b)};
}
MMS_DEV f32pair xpair32(float v) {
  unsigned a = __builtin_bit_cast(unsigned, v), b = a;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return {__builtin_bit_cast(float, a), __builtin_bit_cast(float, b)};
}
MMS_DEV float xsum16(float v) { const f32pair p = xpair16(v); return p.lo + p.hi; }
MMS_DEV float xsum32(float v) { const f32pair p = xpair32(v); return p.lo + p.hi; }
MMS_DEV float xmax16(float v) { const f32pair p = xpair16(v); return fmaxf(p.lo, p.hi); }
MMS_DEV float xmax32(float v) { const f32pair p = xpair32(v); return fmaxf(p.lo, p.hi); }
// sum / max over each 16-lane row
MMS_DEV float row16_sum(float v) {
  v += dpp_f<DPP_ROR8>(v);
  v += dpp_f<DPP_ROR4>(v);
  v += dpp_f<DPP_ROR2>(v);
  return v + dpp_f<DPP_ROR1>(v);
}
MMS_DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<DPP_ROR8>(v));
  v = fmaxf(v, dpp_f<DPP_ROR4>(v));
  v = fmaxf(v, dpp_f<DPP_ROR2>(v));
  return fmaxf(v, dpp_f<DPP_ROR1>(v));
}
MMS_DEV float wave_sum(float v) { return xsum32(xsum16(row16_sum(v))); }
MMS_DEV float wave_max(float v) { return xmax32(xmax16(row16_max(v))); }
MMS_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

MMS_DEV float h2f(h16 x) { return (float)x; }
MMS_DEV h16 f2h(float x) { return (h16)x; }
