// CTC loss (forward + gradient w.r.t. the logits) for the multitask CTC heads.
//
// Semantics: fairseq CtcCriterion (criterions/ctc.py) as the reference's speech_to_unit multitask
// criterion drives it (MultitaskCriterion.get_multitask_loss):
//   lprobs = log_softmax(logits.float()) ; loss = F.ctc_loss(lprobs [T,B,V], targets,
//   input_lengths, target_lengths, blank, reduction="sum", zero_infinity)
// Logits are batch-major fp16 rows (b*T + t) of leading dimension ld (the projection GEMM's
// output); targets int64 [B, tgt_ld] (the first tgt_len[b] entries used).
//
// Layout / schedule: one workgroup per utterance walks time sequentially (the recursion is a
// chain in t); its threads cover the 2S+1 extended labels, two alpha rows double-buffered in LDS.
// The forward stores every alpha row (fp32 [B, T, S2]) for the backward, which runs the beta
// recursion the same way and emits the logits gradient of row t as soon as beta_t is known:
//   dlogit[t][v] = g * (exp(lp[t][v]) - exp(LSE_{s: l'(s)=v}(alpha_t(s) + beta_t(s)) - lp[t][v] + loss))
// (alpha and beta both include the emission at t; PyTorch's ctc_loss backward formula).  The
// per-label log-sum-exp is deterministic and independent of the vocabulary size: the distinct
// labels of the extended sequence are ranked once per utterance (ascending, <= S + 1 of them, in
// LDS, with each position's rank); per time step one thread per distinct label reduces its
// positions in ascending order (max, then sum of exp), and the gradient loop over v finds v's
// rank by binary search.  The summed loss is reduced over utterances in a fixed order.
// All arithmetic fp32; the work is tiny (B x T x 2S) and latency-bound, so it is sized for one
// launch per head per step, not for throughput.
#include <math.h>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

constexpr int CTC_NT = 512;
constexpr float NEG_INF = -INFINITY;

MMS_DEV float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == NEG_INF) return NEG_INF;
  return m + logf(expf(a - m) + expf(b - m));
}

MMS_DEV float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  if (m == NEG_INF) return NEG_INF;
  return m + logf(expf(a - m) + expf(b - m) + expf(c - m));
}

// row log-sum-exp of the logits (fp32), one wave per row
__global__ void ctc_lse_kernel(const h16* __restrict__ logits, long ld, long rows, int V, float* __restrict__ lse) {
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = (gridDim.x * (long)blockDim.x) >> 6;
  for (long r = wave; r < rows; r += nw) {
    const h16* x = logits + r * ld;
    float m = NEG_INF;
    for (int v = lane; v < V; v += 64) m = fmaxf(m, (float)x[v]);
    m = wave_max(m);
    float s = 0.f;
    for (int v = lane; v < V; v += 64) s += expf((float)x[v] - m);
    s = wave_sum(s);
    if (lane == 0) lse[r] = m + logf(s);
  }
}

MMS_DEV int ext_label(const int64_t* tgt, int s, int blank) { return (s & 1) ? (int)tgt[s >> 1] : blank; }

__global__ void __launch_bounds__(CTC_NT) ctc_alpha_kernel(const h16* __restrict__ logits, long ld, int T, int V,
                                                         const float* __restrict__ lse, const int64_t* __restrict__ targets,
                                                         long tgt_ld, const int* __restrict__ in_len,
                                                         const int* __restrict__ tgt_len, int blank, int zero_inf,
                                                         int S2max, float* __restrict__ alpha,
                                                         float* __restrict__ loss_b, float* __restrict__ loss_sum) {
  extern __shared__ float sh[];   // 2 x S2max alpha rows
  const int b = blockIdx.x;
  const int Tb = min(in_len[b], T), Sb = tgt_len[b];
  const int S2 = 2 * Sb + 1;
  const int64_t* tgt = targets + (long)b * tgt_ld;
  float* A = alpha + (long)b * T * S2max;
  const h16* X = logits + (long)b * T * ld;
  const float* Lb = lse + (long)b * T;
  float* cur = sh;
  float* prv = sh + S2max;
  auto lp = [&](int t, int v) { return (float)X[(long)t * ld + v] - Lb[t]; };
  for (int s = threadIdx.x; s < S2; s += blockDim.x) {
    const float a = (s < 2 && Tb > 0) ? lp(0, ext_label(tgt, s, blank)) : NEG_INF;
    cur[s] = a;
    A[s] = a;
  }
  __syncthreads();
  for (int t = 1; t < Tb; ++t) {
    float* tmp = prv; prv = cur; cur = tmp;
    for (int s = threadIdx.x; s < S2; s += blockDim.x) {
      const int l = ext_label(tgt, s, blank);
      float a = prv[s];
      if (s >= 1) a = lse2(a, prv[s - 1]);
      if (s >= 2 && l != blank && l != ext_label(tgt, s - 2, blank)) a = lse2(a, prv[s - 2]);
      a = (a == NEG_INF) ? NEG_INF : a + lp(t, l);
      cur[s] = a;
      A[(long)t * S2max + s] = a;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float ll = NEG_INF;
    if (Tb > 0) ll = (S2 >= 2) ? lse2(cur[S2 - 1], cur[S2 - 2]) : cur[S2 - 1];
    float loss = -ll;
    if (!isfinite(loss) && zero_inf) loss = 0.f;
    loss_b[b] = loss;
  }
}

// loss_sum[0] += sum_b loss_b[b], one wave, fixed order (bit-reproducible; no float atomics)
__global__ void ctc_loss_sum_kernel(const float* __restrict__ loss_b, int B, float* __restrict__ loss_sum) {
  float s = 0.f;
  for (int b = threadIdx.x; b < B; b += 64) s += loss_b[b];
  s = wave_sum(s);
  if (threadIdx.x == 0) loss_sum[0] += s;
}

__global__ void __launch_bounds__(CTC_NT) ctc_beta_grad_kernel(const h16* __restrict__ logits, long ld, int T, int V,
                                                             const float* __restrict__ lse, const int64_t* __restrict__ targets,
                                                             long tgt_ld, const int* __restrict__ in_len,
                                                             const int* __restrict__ tgt_len, int blank,
                                                             int S2max, const float* __restrict__ alpha,
                                                             const float* __restrict__ loss_b,
                                                             const float* __restrict__ grad_scale, h16* __restrict__ dlogits,
                                                             long ldd) {
  extern __shared__ float sh[];   // 2 x S2max beta rows | S2max ranks (int) | S2max labels (int) | S2max gammas
  const int b = blockIdx.x;
  const int Tb = min(in_len[b], T), Sb = tgt_len[b];
  const int S2 = 2 * Sb + 1;
  const int64_t* tgt = targets + (long)b * tgt_ld;
  const float* A = alpha + (long)b * T * S2max;
  const h16* X = logits + (long)b * T * ld;
  const float* Lb = lse + (long)b * T;
  h16* D = dlogits + (long)b * T * ldd;
  float* cur = sh;
  float* nxt = sh + S2max;
  int* own = reinterpret_cast<int*>(sh + 2 * S2max);   // [S2] rank of position s's label
  int* lab = own + S2max;                              // [U] distinct labels, ascending
  float* gam = reinterpret_cast<float*>(lab + S2max);  // [U] log-sum-exp of alpha + beta per label
  __shared__ int U;
  const float g = grad_scale[0];
  auto lp = [&](int t, int v) { return (float)X[(long)t * ld + v] - Lb[t]; };
  // distinct labels: own[s] = 1 at a label's first position, then ranks by label value
  if (threadIdx.x == 0) U = 0;
  for (int s = threadIdx.x; s < S2; s += blockDim.x) {
    const int l = ext_label(tgt, s, blank);
    int first = 1;
    for (int q = 0; q < s && first; ++q) first = ext_label(tgt, q, blank) != l;
    own[s] = first;
  }
  __syncthreads();
  for (int s = threadIdx.x; s < S2; s += blockDim.x) {
    if (!own[s]) continue;
    const int l = ext_label(tgt, s, blank);
    int r = 0;
    for (int q = 0; q < S2; ++q) r += (own[q] && ext_label(tgt, q, blank) < l) ? 1 : 0;
    lab[r] = l;
    atomicAdd(&U, 1);
  }
  __syncthreads();
  const int nU = U;
  auto rank_of = [&](int v) {          // index of v in lab[0, nU) or -1
    int lo = 0, hi = nU - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      const int x = lab[mid];
      if (x == v) return mid;
      if (x < v) lo = mid + 1; else hi = mid - 1;
    }
    return -1;
  };
  for (int s = threadIdx.x; s < S2; s += blockDim.x) own[s] = rank_of(ext_label(tgt, s, blank));
  // padded time steps and padded columns: zero gradient
  for (int t = Tb; t < T; ++t)
    for (int v = threadIdx.x; v < (int)ldd; v += blockDim.x) D[(long)t * ldd + v] = (h16)0.f;
  // an impossible alignment (loss = +inf, or zeroed by zero_infinity): gradient 0 (torch zero_infinity)
  float lastA = NEG_INF;
  if (Tb > 0) {
    const float* Al = A + (long)(Tb - 1) * S2max;
    lastA = (S2 >= 2) ? lse2(Al[S2 - 1], Al[S2 - 2]) : Al[S2 - 1];
  }
  const bool impossible = !(lastA > NEG_INF);
  (void)loss_b;
  __syncthreads();
  for (int t = Tb - 1; t >= 0; --t) {
    float* tmp = nxt; nxt = cur; cur = tmp;
    for (int s = threadIdx.x; s < S2; s += blockDim.x) {
      const int l = ext_label(tgt, s, blank);
      float bt;
      if (t == Tb - 1) {
        bt = (s >= S2 - 2) ? lp(t, l) : NEG_INF;
      } else {
        bt = nxt[s];
        if (s + 1 < S2) bt = lse2(bt, nxt[s + 1]);
        if (s + 2 < S2 && l != blank && l != ext_label(tgt, s + 2, blank)) bt = lse2(bt, nxt[s + 2]);
        bt = (bt == NEG_INF) ? NEG_INF : bt + lp(t, l);
      }
      cur[s] = bt;
    }
    __syncthreads();
    const float* At = A + (long)t * S2max;
    for (int j = threadIdx.x; j < nU; j += blockDim.x) {
      float m = NEG_INF;
      for (int s = 0; s < S2; ++s)
        if (own[s] == j) m = fmaxf(m, At[s] + cur[s]);
      float acc = 0.f;
      if (m > NEG_INF)
        for (int s = 0; s < S2; ++s)
          if (own[s] == j) {
            const float ab = At[s] + cur[s];
            if (ab > NEG_INF) acc += expf(ab - m);
          }
      gam[j] = (m > NEG_INF) ? m + logf(acc) : NEG_INF;
    }
    __syncthreads();
    for (int v = threadIdx.x; v < (int)ldd; v += blockDim.x) {
      float d = 0.f;
      if (v < V && !impossible) {
        const float lpv = lp(t, v);
        d = expf(lpv);
        const int j = rank_of(v);
        if (j >= 0 && gam[j] > NEG_INF) d -= expf(gam[j] - lpv - lastA);
        d *= g;
      }
      D[(long)t * ldd + v] = (h16)d;
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int mms2ut_ctc_workspace_floats(int B, int T, int max_tgt_len, int64_t* n) {
  MMS_REQUIRE(n != nullptr && B >= 0 && T >= 0 && max_tgt_len >= 0, "ctc_workspace: bad args");
  const long S2 = 2L * max_tgt_len + 1;
  *n = (long)B * T + (long)B * T * S2 + B;   // lse | alpha | per-utterance losses
  return 0;
}

extern "C" int mms2ut_ctc_loss_fwd(const h16* logits, int64_t ld, int B, int T, int V, const int64_t* targets,
                                   int64_t tgt_ld, int max_tgt_len, const int* in_len, const int* tgt_len, int blank,
                                   int zero_infinity, float* work, float* loss_sum, hipStream_t s) {
  MMS_REQUIRE(V > 0 && ld >= V && blank >= 0 && blank < V && max_tgt_len >= 0 && tgt_ld >= max_tgt_len,
              "ctc_loss: bad shapes (V=%d ld=%ld blank=%d S=%d)", V, (long)ld, blank, max_tgt_len);
  const int S2 = 2 * max_tgt_len + 1;
  MMS_REQUIRE((size_t)5 * S2 * sizeof(float) <= 64 * 1024, "ctc_loss: target too long (%d labels, max %d)",
              max_tgt_len, (int)((64 * 1024 / (5 * sizeof(float)) - 1) / 2));
  if (B == 0 || T == 0) return 0;
  float* lse = work;
  float* alpha = work + (long)B * T;
  float* loss_b = alpha + (long)B * T * S2;
  const long rows = (long)B * T;
  hipLaunchKernelGGL(ctc_lse_kernel, dim3((unsigned)std::min<long>((rows + 3) / 4, 4096)), dim3(256), 0, s,
                     logits, (long)ld, rows, V, lse);
  hipLaunchKernelGGL(ctc_alpha_kernel, dim3(B), dim3(CTC_NT), 2 * S2 * sizeof(float), s, logits, (long)ld, T, V,
                     lse, targets, (long)tgt_ld, in_len, tgt_len, blank, zero_infinity, S2, alpha, loss_b, loss_sum);
  hipLaunchKernelGGL(ctc_loss_sum_kernel, dim3(1), dim3(64), 0, s, loss_b, B, loss_sum);
  return mms::check_launch("ctc_loss_fwd");
}

extern "C" int mms2ut_ctc_loss_bwd(const h16* logits, int64_t ld, int B, int T, int V, const int64_t* targets,
                                   int64_t tgt_ld, int max_tgt_len, const int* in_len, const int* tgt_len, int blank,
                                   const float* work, const float* grad_scale, h16* dlogits, int64_t ldd,
                                   hipStream_t s) {
  MMS_REQUIRE(ldd >= V && ldd % 4 == 0, "ctc_loss_bwd: ldd must be >= V and a multiple of 4");
  const int S2 = 2 * max_tgt_len + 1;
  const size_t lds = 5 * (size_t)S2 * sizeof(float);   // independent of the vocabulary size
  MMS_REQUIRE(lds <= 64 * 1024, "ctc_loss_bwd: target too long for LDS (%d labels, max %d)", max_tgt_len,
              (int)((64 * 1024 / (5 * sizeof(float)) - 1) / 2));
  if (B == 0 || T == 0) return 0;
  const float* lse = work;
  const float* alpha = work + (long)B * T;
  const float* loss_b = alpha + (long)B * T * S2;
  hipLaunchKernelGGL(ctc_beta_grad_kernel, dim3(B), dim3(CTC_NT), lds, s, logits, (long)ld, T, V, lse, targets,
                     (long)tgt_ld, in_len, tgt_len, blank, S2, alpha, loss_b, grad_scale, dlogits, (long)ldd);
  return mms::check_launch("ctc_loss_bwd");
}
