// Microbenchmark: issue cost of 32-bit integer multiplies vs adds on gfx950 (one wave per SIMD,
// 8 independent chains).  Prints cycles per instruction per wave.  hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int OP>
__global__ void k(unsigned* out, unsigned seed, long long* cyc) {
  unsigned x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i;
  const unsigned c = 0x7feb352dU;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 1024; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) x[i] = x[i] * c;                                     // v_mul_lo_u32
      else if (OP == 1) x[i] = x[i] + c;                                // v_add_u32
      else if (OP == 2) x[i] = __umul24(x[i], c);       // v_mul_u32_u24
      else if (OP == 3) x[i] = x[i] ^ (x[i] >> 15);                     // shift + xor
      else x[i] = (unsigned)(((unsigned long long)x[i] * c) >> 32) ^ x[i];  // v_mul_hi_u32
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  unsigned* out; long long* cyc;
  hipMalloc(&out, 256 * 64 * 4); hipMalloc(&cyc, 8);
  const char* names[] = {"v_mul_lo_u32", "v_add_u32", "v_mul_u32_u24", "lshr+xor (2 instr)", "v_mul_hi_u32 + xor (2 instr)"};
  for (int op = 0; op < 5; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (op) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(64), 0, 0, out, 1u, cyc); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(64), 0, 0, out, 1u, cyc); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(64), 0, 0, out, 1u, cyc); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(64), 0, 0, out, 1u, cyc); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(64), 0, 0, out, 1u, cyc); break;
      }
      hipDeviceSynchronize();
    }
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-30s %.2f cycles per wave-instruction step (8192 per wave)\n", names[op], (double)c / 8192.0);
  }
  return 0;
}
