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
MMS_DEV uint32_t mms_hash(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed ^ (ctr * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
// keep with probability 1-p: hash >= p * 2^32
MMS_DEV bool mms_keep(uint64_t seed, uint64_t ctr, uint32_t thresh) {
  return mms_hash(seed, ctr) >= thresh;
}
static inline uint32_t mms_drop_thresh(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) return 4294967295u;
  return (uint32_t)t;
}

// ------------------------------------------------------------------------------------------
// wave64 reductions
// ------------------------------------------------------------------------------------------
MMS_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MMS_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
MMS_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

MMS_DEV float h2f(h16 x) { return (float)x; }
MMS_DEV h16 f2h(float x) { return (h16)x; }
