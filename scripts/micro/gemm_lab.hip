// GEMM lab: isolated A/B of candidate NT kernels against the library's dispatch on the step's
// shapes (random fp16, warm, HIP events, interleaved rounds), with a bitwise comparison of every
// candidate's C against the library's.  Build: scripts/micro/build_gemm_lab.sh; run on the box:
//   scripts/micro/gemm_lab [reps]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../multimodal-s2ut_amd/csrc/gemm_common.h"

#include "lab_gemm_wide.h"
#include "lab_gemm_persist.h"
#include "lab_gemm_stagger.h"


// ---------------------------------------------------------------------------------------------
// Experiment: persistent form of gemm_tall_kernel (2 blocks per CU, static tile walk) with
// per-block roles: ROLE 1 = blocks of the first half of the grid (likely the first block on each
// CU) run at a higher wave priority, so the two blocks of a CU drift apart and one's epilogue
// runs under the other's k-loop.  ROLE 0 = same priority (persistence alone).
// ---------------------------------------------------------------------------------------------
__device__ unsigned long long* g_lab_hw = nullptr;

template <int EPI, int FRT, int ROLE>
__global__ void __launch_bounds__(NT, 2) gemm_tallp_kernel(GemmP P, int tiles_m, int tiles_n, int total) {
  constexpr int BMT = 32 * FRT, TILE_T = BMT * 64 * 2;
  constexpr int SMEM = 2 * (TILE_T + TILE_BYTES) > 4 * 64 * 64 * 4 ? 2 * (TILE_T + TILE_BYTES) : 4 * 64 * 64 * 4;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  if (g_lab_hw && threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));
    g_lab_hw[blockIdx.x] = ((unsigned long long)xcc << 32) | hw;
  }
  const bool lead = ROLE == 1 && (int)blockIdx.x < (int)gridDim.x / 2;
  const int pr_hi = lead ? 3 : 1, pr_lo = lead ? 2 : 0;
  const long a_ext = ((long)(P.M - 1) * P.lda + P.K) * 2;
  const long b_ext = ((long)(P.N - 1) * P.ldb + P.K) * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)P.A, (short)0, (int)a_ext, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)P.B, (short)0, (int)b_ext, 0x00020000);
  const int nk = P.K / BK;
  for (int lin = blockIdx.x; lin < total; lin += gridDim.x) {
    if (lin != (int)blockIdx.x) __syncthreads();
    int z, tm, tn;
    tile_coords(lin, tiles_m, tiles_n, total, z, tm, tn, P.group_m);
    const int bm = tm * BMT, bn = tn * BN;
#define SA(s) (smem + (s) * (TILE_T + TILE_BYTES))
#define SB(s) (SA(s) + TILE_T)
    auto dma_a = [&](char* lds, int k0) {
#pragma unroll
      for (int x = 0; x < FRT; ++x) {
        const int ins = wid * FRT + x;
        const int row = ins * 8 + (lane >> 3), c = (lane & 7) ^ (row & 7);
        const int voff = (int)(((long)(bm + row) * P.lda + k0 + c * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(lds + ins * 1024), 16, voff, 0, 0, 0);
      }
    };
    f32x4 acc[FRT][4];
#pragma unroll
    for (int i = 0; i < FRT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    dma_a(SA(0), 0);
    dma_tile<true>(rb, SB(0), P.ldb, bn, 0, wid, lane);
    for (int kt = 0; kt < nk; ++kt) {
      wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      const int cur = kt & 1;
      if (kt + 1 < nk) {
        dma_a(SA(cur ^ 1), (kt + 1) * BK);
        dma_tile<true>(rb, SB(cur ^ 1), P.ldb, bn, (kt + 1) * BK, wid, lane);
      }
      h16x8 fa2[2][FRT], fb2[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < FRT; ++i) fa2[kk][i] = read_frag<true>(SA(cur), wm * 16 * FRT + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb2[kk][j] = read_frag<true>(SB(cur), wn * 64 + j * 16, kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (ROLE == 1) { if (lead) __builtin_amdgcn_s_setprio(3); else __builtin_amdgcn_s_setprio(1); }
        else __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FRT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb2[kk][j], fa2[kk][i], acc[i][j], 0, 0, 0);
        if (ROLE == 1) { if (lead) __builtin_amdgcn_s_setprio(2); else __builtin_amdgcn_s_setprio(0); }
        else __builtin_amdgcn_s_setprio(0);
      }
    }
#undef SA
#undef SB
    (void)pr_hi; (void)pr_lo;
    __syncthreads();
    constexpr int WR = 16 * FRT, F1 = FRT < 4 ? FRT : 4;
    staged_epilogue<EPI, F1>(P, smem, reinterpret_cast<const f32x4(&)[F1][4]>(acc[0]), bm + (WR - 64) * wm, bn, wm,
                             wn, wid, lane, P.C, P.aux);
    if constexpr (FRT > 4) {
      __syncthreads();
      staged_epilogue<EPI, FRT - 4>(P, smem, reinterpret_cast<const f32x4(&)[FRT - 4][4]>(acc[4]),
                                    bm + (WR - 64) * wm + 64, bn, wm, wn, wid, lane, P.C, P.aux);
    }
  }
}

template <int FRT, int ROLE>
static int launch_tallp_t(int epi, const GemmP& P, hipStream_t s, int grid_cap) {
  constexpr int BMT = 32 * FRT;
  const int tm = (P.M + BMT - 1) / BMT, tn = (P.N + 127) / 128, total = tm * tn;
  const int grid = std::min(total, grid_cap);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((gemm_tallp_kernel<E, FRT, ROLE>), dim3(grid), dim3(NT), 0, s, P, tm, tn, total); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_RELU_DROP_BWD)
#undef CASE
    default: return 1;
  }
  return hipGetLastError() != hipSuccess;
}
template <int FRT, bool DEFER>
static int launch_persist_t(int epi, GemmP P, hipStream_t s) {
  constexpr int BMT = 32 * FRT;
  const int tm = (P.M + BMT - 1) / BMT, tn = (P.N + 127) / 128, total = tm * tn;
  const int grid = std::min(total, 512);
  switch (epi) {
#define CASE(E) case E: hipLaunchKernelGGL((mmsp::gemm_persist_kernel<E, FRT, DEFER>), dim3(grid), dim3(NT), 0, s, P, tm, tn, total); break;
    CASE(MMS_EPI_F16) CASE(MMS_EPI_RELU_DROP) CASE(MMS_EPI_DROP_RESID) CASE(MMS_EPI_RELU_DROP_BWD)
#undef CASE
    default: return 1;
  }
  return hipGetLastError() != hipSuccess;
}
static int launch_persist(int epi, int bm, int defer, const GemmP& P, hipStream_t s) {
  if (bm == 192) return defer ? launch_persist_t<6, true>(epi, P, s) : launch_persist_t<6, false>(epi, P, s);
  if (bm == 160) return defer ? launch_persist_t<5, true>(epi, P, s) : launch_persist_t<5, false>(epi, P, s);
  if (bm == 128) return defer ? launch_persist_t<4, true>(epi, P, s) : launch_persist_t<4, false>(epi, P, s);
  return 1;
}
static int launch_tallp(int epi, int bm, int role, const GemmP& P, hipStream_t s) {
  if (bm == 192) return role ? launch_tallp_t<6, 1>(epi, P, s, 512) : launch_tallp_t<6, 0>(epi, P, s, 512);
  if (bm == 160) return role ? launch_tallp_t<5, 1>(epi, P, s, 512) : launch_tallp_t<5, 0>(epi, P, s, 512);
  if (bm == 128) return role ? launch_tallp_t<4, 1>(epi, P, s, 512) : launch_tallp_t<4, 0>(epi, P, s, 512);
  return 1;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void fill_kernel(h16* p, long n, uint32_t seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint32_t h = mms_mix32((uint32_t)i * 2654435761U ^ mms_mix32(seed + (uint32_t)(i >> 32)));
    p[i] = (h16)(((float)(h & 0xffffff) / 8388608.f - 1.f) * scale);
  }
}

static void fill(h16* p, long n, uint32_t seed, float scale) {
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, p, n, seed, scale);
  CK(hipGetLastError());
}

struct Shape {
  const char* name;
  int M, N, K, epi;
  float p;
};

static mms2ut_gemm_args make_args(const Shape& s, h16* A, h16* B, h16* C, h16* bias, h16* aux) {
  mms2ut_gemm_args a;
  memset(&a, 0, sizeof(a));
  a.A = A; a.B = B; a.C = C;
  a.M = s.M; a.N = s.N; a.K = s.K;
  a.a_kcontig = 1; a.b_kcontig = 1;
  a.lda = s.K; a.ldb = s.K; a.ldc = s.N;
  a.batch = 1; a.bdiv = 1; a.splitk = 1;
  a.epi = s.epi;
  a.alpha = 1.f;
  a.bias = (s.epi == MMS_EPI_RELU_DROP_BWD) ? nullptr : bias;
  const bool needs_aux = s.epi == MMS_EPI_DROP_RESID || s.epi == MMS_EPI_RELU_DROP_BWD;
  a.aux = needs_aux ? aux : nullptr;
  a.ldaux = s.N;
  a.dropout_p = s.p;
  a.seed = 1234;
  a.offset = 0;
  a.ld_rng = s.N;
  return a;
}

static GemmP make_p(const mms2ut_gemm_args& a) {
  GemmP P{};
  P.A = a.A; P.B = a.B; P.C = a.C;
  P.M = a.M; P.N = a.N; P.K = a.K;
  P.lda = a.lda; P.ldb = a.ldb; P.ldc = a.ldc;
  P.bdiv = 1; P.splitk = 1; P.kchunk = a.K;
  P.alpha = a.alpha; P.bias = a.bias;
  P.aux = a.aux; P.ldaux = a.ldaux;
  P.out2 = a.out2; P.ldo2 = a.ldo2;
  P.p = a.dropout_p; P.thresh = mms_drop_thresh(a.dropout_p); P.seed = a.seed; P.offset = a.offset;
  P.ld_rng = a.ld_rng;
  P.vec16 = 1;
  P.group_m = 8;
  return P;
}

typedef int (*LaunchFn)(const mms2ut_gemm_args&, hipStream_t);

struct Variant {
  const char* name;
  int kind;   // 0 library default, 1 library 128x128 only, 2 wide candidate, 3 wide without epilogue,
              // 4 persistent tall (var = role)
  int bm, var;
};

static int run_variant(const Variant& v, const mms2ut_gemm_args& a, hipStream_t s) {
  if (v.kind == 0) { mms2ut_gemm_set_tall(1); return mms2ut_gemm_f16(&a, s); }
  if (v.kind == 1) { mms2ut_gemm_set_tall(0); int rc = mms2ut_gemm_f16(&a, s); mms2ut_gemm_set_tall(1); return rc; }
  GemmP P = make_p(a);
  if (v.kind == 4) return launch_tallp(a.epi, v.bm, v.var, P, s);
  if (v.kind == 5) return launch_persist(a.epi, v.bm, v.var, P, s);
  if (v.kind == 6) return mmst::launch_stag(a.epi, v.bm, v.var, P, s);
  if (v.kind == 7) return mmst::launch_pf(a.epi, v.bm, P, s);
  return mmsw::launch_wide(a.epi, v.bm, v.var, P, s, v.kind == 3);
}

int main(int argc, char** argv) {
#ifdef MMS_LAB_NOSTORE
  printf("# build: staged epilogue without its C stores (MMS_LAB_NOSTORE)\n");
#endif
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const int only = argc > 2 ? atoi(argv[2]) : -1;
  std::vector<Shape> shapes = {
      {"sq8192", 8192, 8192, 8192, MMS_EPI_F16, 0.f},
      {"fc1_fwd", 10000, 3072, 768, MMS_EPI_RELU_DROP, 0.1f},
      {"fc1_plain", 10000, 3072, 768, MMS_EPI_F16, 0.f},
      {"fc1_relu", 10000, 3072, 768, MMS_EPI_RELU_DROP, 0.f},
      {"fc1_resid", 10000, 3072, 768, MMS_EPI_DROP_RESID, 0.1f},
      {"qkv_fwd", 10000, 2304, 768, MMS_EPI_F16, 0.f},
      {"fc2_dgrad", 10000, 3072, 768, MMS_EPI_RELU_DROP_BWD, 0.1f},
      {"out_proj", 10000, 768, 768, MMS_EPI_DROP_RESID, 0.1f},
      {"fc2_fwd", 10000, 768, 3072, MMS_EPI_DROP_RESID, 0.1f},
      {"qkv_dgrad", 10000, 768, 2304, MMS_EPI_F16, 0.f},
      {"dec_fc1", 12100, 3072, 768, MMS_EPI_RELU_DROP, 0.1f},
      {"dec_qkv", 12100, 2304, 768, MMS_EPI_F16, 0.f},
      {"dec_fc2", 12100, 768, 3072, MMS_EPI_DROP_RESID, 0.1f},
  };
  std::vector<Variant> vars = {
      {"lib", 0, 0, 0},
      {"st192", 6, 192, 0},
      {"pf192", 7, 192, 0},
      {"st128", 6, 128, 0},
      {"pf128", 7, 128, 0},
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (size_t si = 0; si < shapes.size(); ++si) {
    if (only >= 0 && (int)si != only) continue;
    const Shape& s = shapes[si];
    h16 *A, *B, *bias, *aux, *Cref, *C;
    CK(hipMalloc(&A, (size_t)s.M * s.K * 2));
    CK(hipMalloc(&B, (size_t)s.N * s.K * 2));
    CK(hipMalloc(&bias, (size_t)s.N * 2));
    CK(hipMalloc(&aux, (size_t)s.M * s.N * 2));
    CK(hipMalloc(&Cref, (size_t)s.M * s.N * 2));
    CK(hipMalloc(&C, (size_t)s.M * s.N * 2));
    fill(A, (long)s.M * s.K, 11 + si, 0.5f);
    fill(B, (long)s.N * s.K, 23 + si, 0.05f);
    fill(bias, s.N, 37 + si, 0.1f);
    fill(aux, (long)s.M * s.N, 41 + si, 1.0f);
    CK(hipDeviceSynchronize());
    mms2ut_gemm_args a = make_args(s, A, B, Cref, bias, aux);
    if (mms2ut_gemm_f16(&a, st)) { fprintf(stderr, "ref: %s\n", mms2ut_last_error()); return 1; }
    CK(hipStreamSynchronize(st));
    std::vector<uint16_t> href((size_t)s.M * s.N), hc((size_t)s.M * s.N);
    CK(hipMemcpy(href.data(), Cref, href.size() * 2, hipMemcpyDeviceToHost));
    const double tf = 2.0 * s.M * s.N * (double)s.K / 1e12;
    std::vector<std::vector<float>> times(vars.size());
    std::vector<long> mism(vars.size(), -1);
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      a.C = C;
      CK(hipMemsetAsync(C, 0xff, (size_t)s.M * s.N * 2, st));
      if (run_variant(vars[vi], a, st)) { fprintf(stderr, "%s: launch failed\n", vars[vi].name); mism[vi] = -2; continue; }
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
      long m = 0;
      for (size_t i = 0; i < hc.size(); ++i) m += hc[i] != href[i];
      mism[vi] = m;
    }
    if (si == 99) {   // co-residency census of the persistent grid (512 blocks)
      unsigned long long* d_hw;
      CK(hipMalloc(&d_hw, 512 * 8));
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_lab_hw), &d_hw, sizeof(d_hw)));
      GemmP P = make_p(a);
      launch_tallp(a.epi, 192, 1, P, st);
      CK(hipStreamSynchronize(st));
      unsigned long long* z = nullptr;
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_lab_hw), &z, sizeof(z)));
      std::vector<unsigned long long> hw(512);
      CK(hipMemcpy(hw.data(), d_hw, 512 * 8, hipMemcpyDeviceToHost));
      int paired_half = 0, pairs = 0, maxocc = 0;
      std::vector<int> seen(512, 0);
      for (int b = 0; b < 512; ++b) {
        if (seen[b]) continue;
        const unsigned long long key = (hw[b] >> 32 << 32) | (hw[b] & 0xff00ULL);
        std::vector<int> grp;
        for (int c = b; c < 512; ++c)
          if (!seen[c] && ((hw[c] >> 32 << 32) | (hw[c] & 0xff00ULL)) == key) { grp.push_back(c); seen[c] = 1; }
        maxocc = std::max(maxocc, (int)grp.size());
        if (grp.size() == 2) { ++pairs; if ((grp[0] < 256) != (grp[1] < 256)) ++paired_half; }
        if (b < 24) {
          printf("  cu key %llx:", key);
          for (int c : grp) printf(" %d(w%llu)", c, hw[c] & 15ULL);
          printf("\n");
        }
      }
      printf("census: %d CU pairs, %d of them one block from each half of the grid, max %d blocks per CU\n", pairs,
             paired_half, maxocc);
      CK(hipFree(d_hw));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 3; ++round) {
      for (size_t vi = 0; vi < vars.size(); ++vi) {
        if (mism[vi] == -2) continue;
        a.C = C;
        for (int w = 0; w < 3; ++w) run_variant(vars[vi], a, st);
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; ++r) run_variant(vars[vi], a, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        times[vi].push_back(ms * 1e3f / reps);
      }
    }
    printf("%-10s M=%5d N=%5d K=%5d epi=%d\n", s.name, s.M, s.N, s.K, s.epi);
    {
      unsigned long long* d_clk;
      const int maxb = 8192;
      CK(hipMalloc(&d_clk, (size_t)maxb * 32));
      for (size_t vi = 0; vi < vars.size(); ++vi) {
        if (vars[vi].kind < 2 || vars[vi].kind > 3) continue;
        CK(hipMemset(d_clk, 0, (size_t)maxb * 32));
        for (int w = 0; w < 30; ++w) run_variant(vars[vi], a, st);   // warm the clock governor
        CK(hipMemcpyToSymbol(HIP_SYMBOL(mmsw::g_w_clk), &d_clk, sizeof(d_clk)));
        run_variant(vars[vi], a, st);
        CK(hipStreamSynchronize(st));
        unsigned long long* z = nullptr;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(mmsw::g_w_clk), &z, sizeof(z)));
        std::vector<unsigned long long> h((size_t)maxb * 4);
        CK(hipMemcpy(h.data(), d_clk, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> mhz, span;
        for (int b = 0; b < maxb; ++b) {
          const unsigned long long c0 = h[4 * b], r0 = h[4 * b + 1], c1 = h[4 * b + 2], r1 = h[4 * b + 3];
          if (r1 <= r0) continue;
          mhz.push_back((double)(c1 - c0) / (double)(r1 - r0) * 100.0);
          span.push_back((double)(r1 - r0) / 100.0);
        }
        if (mhz.empty()) continue;
        std::sort(mhz.begin(), mhz.end());
        std::sort(span.begin(), span.end());
        printf("    clock %-12s %7.0f MHz (blocks %zu), loop span median %.1f us\n", vars[vi].name, mhz[mhz.size() / 2],
               mhz.size(), span[span.size() / 2]);
      }
      CK(hipFree(d_clk));
    }
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      if (times[vi].empty()) { printf("    %-12s FAILED\n", vars[vi].name); continue; }
      std::vector<float> t = times[vi];
      std::sort(t.begin(), t.end());
      printf("    %-12s %8.1f us (min %8.1f) %6.0f TF  mismatches %ld\n", vars[vi].name, t[t.size() / 2], t[0],
             tf / t[t.size() / 2] * 1e6, mism[vi]);
    }
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(bias)); CK(hipFree(aux)); CK(hipFree(Cref)); CK(hipFree(C));
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  }
  return 0;
}
