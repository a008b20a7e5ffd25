// Probe: what __builtin_amdgcn_permlane16_swap / permlane32_swap return on gfx950 (lane l: a = l,
// b = 100 + l), and the reduction form (one value on both operands, results added): through the
// builtin the compiler adds the first result to itself; through inline asm the sum is right.
// Prints per-lane values.  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned a = l, b = 100 + l;
  asm volatile("" : "+v"(a), "+v"(b));
  const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  unsigned c = l, d = 100 + l;
  asm volatile("" : "+v"(c), "+v"(d));
  const auto s = __builtin_amdgcn_permlane32_swap(c, d, false, false);
  out[128 + l] = s[0];
  out[192 + l] = s[1];
  // the reduction form: one value on both operands (second one made opaque), results added
  float v = (float)l;
  unsigned x = __builtin_bit_cast(unsigned, v), y = x;
  asm volatile("" : "+v"(y));
  const auto t = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[256 + l] = (unsigned)(__builtin_bit_cast(float, t[0]) + __builtin_bit_cast(float, t[1]));
  // the same through inline asm (csrc/common.h xpair16)
  unsigned x2 = __builtin_bit_cast(unsigned, v), y2 = x2;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x2), "+v"(y2));
  out[320 + l] = (unsigned)(__builtin_bit_cast(float, x2) + __builtin_bit_cast(float, y2));
}
int main() {
  unsigned* d; hipMalloc(&d, 384 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[384]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[6] = {"p16 r0", "p16 r1", "p32 r0", "p32 r1", "p16 sum(v,v) builtin", "p16 sum(v,v) asm"};
  for (int t = 0; t < 6; ++t) { printf("%s:", nm[t]); for (int l = 0; l < 64; l += 4) printf(" %u", h[64 * t + l]); printf("\n"); }
  return 0;
}
