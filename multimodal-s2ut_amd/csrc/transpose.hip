// Batched fp16 matrix transpose: the weight images W^T that let every dgrad GEMM read both
// operands K-contiguous (ds_read_b128 fragments instead of transposed reads; round-2 A/B, scripts/gemm_ab.py in git history:
// 13-20 % faster on the step's dgrad shapes).  One launch refreshes every registered matrix after
// each optimizer update; it runs on the side stream beside the next forward.
//
// Each 256-thread block moves one 64x64 tile: 16-B row loads into an LDS tile padded to 72 halves
// per row, then each thread gathers 8 consecutive source rows of one column and writes them as one
// 16-B store of the transposed row.
#include "common.h"
#include "../../include/mms2ut.h"

namespace {

constexpr int TT = 64, TLD = TT + 8;

__global__ void __launch_bounds__(256) transpose_batch_kernel(const h16* __restrict__ src, h16* __restrict__ dst,
                                                              const mms2ut_transpose_desc* __restrict__ d, int n) {
  __shared__ __attribute__((aligned(16))) h16 tile[TT * TLD];
  const int b = blockIdx.x;
  // matrix of this block: the descriptors are sorted by first tile; binary search for the last one
  // with tile0 <= b (a linear scan is a chain of up to n dependent scalar loads per block)
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].tile0 <= b) lo = mid; else hi = mid - 1;
  }
  const int i = lo;
  const mms2ut_transpose_desc D = d[i];
  const int tiles_c = (D.cols + TT - 1) / TT;
  const int t = b - D.tile0, r0 = (t / tiles_c) * TT, c0 = (t % tiles_c) * TT;
  const h16* S = src + D.src;
  h16* T = dst + D.dst;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = threadIdx.x + 256 * k, r = id >> 3, c = (id & 7) * 8;
    s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + r < D.rows && c0 + c < D.cols) v = *reinterpret_cast<const s16x8*>(S + (long)(r0 + r) * D.cols + c0 + c);
    *reinterpret_cast<s16x8*>(tile + r * TLD + c) = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = threadIdx.x + 256 * k, c = id >> 3, r = (id & 7) * 8;  // output row c, cols r..r+7
    if (c0 + c < D.cols && r0 + r < D.rows) {
      h16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = tile[(r + e) * TLD + c];
      *reinterpret_cast<h16x8*>(T + (long)(c0 + c) * D.rows + r0 + r) = o;
    }
  }
}

}  // namespace

extern "C" int mms2ut_transpose_batch(const mms2ut_half* src, mms2ut_half* dst, const mms2ut_transpose_desc* descs,
                                      int n, int total_tiles, hipStream_t s) {
  MMS_REQUIRE(src && dst && descs && n > 0 && total_tiles > 0, "transpose_batch: bad arguments");
  MMS_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "transpose_batch: buffers must be 16-B aligned");
  hipLaunchKernelGGL(transpose_batch_kernel, dim3(total_tiles), dim3(256), 0, s, src, dst, descs, n);
  return mms::check_launch("transpose_batch");
}
