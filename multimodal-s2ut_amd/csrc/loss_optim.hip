// Label-smoothed cross entropy (fused fp32 log-softmax) and the FP16Optimizer/Adam update.
#include <algorithm>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

// one wave per row of logits; V <= 64*4*CPL
template <int CPL>
__global__ void __launch_bounds__(256) ls_xent_fwd_kernel(const h16* __restrict__ z, long ld,
                                                          const int64_t* __restrict__ target, long rows,
                                                          int V, float eps, int pad, float* __restrict__ lse_out,
                                                          float* __restrict__ part) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float loss = 0.f, nll = 0.f;
  // grid-stride over a bounded grid (<= MMS_LS_XENT_PARTS blocks); each block leaves its {loss, nll}
  // partial, summed in block order by ls_xent_sum_kernel (no float atomics: the loss is
  // bit-reproducible)
  for (long row = (long)blockIdx.x * 4 + w; row < rows; row += (long)gridDim.x * 4) {
    const h16* zr = z + row * ld;
    float v[CPL][4];
    float mx = -INFINITY, sum = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int j0 = (lane + c * 64) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[c][e] = -INFINITY;
      if (j0 < V) {
        h16x4 t = *reinterpret_cast<const h16x4*>(zr + j0);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (j0 + e < V) { v[c][e] = (float)t[e]; mx = fmaxf(mx, v[c][e]); sum += v[c][e]; }
      }
    }
    mx = wave_max(mx);
    sum = wave_sum(sum);
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) se += (v[c][e] == -INFINITY) ? 0.f : __expf(v[c][e] - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    if (lane == 0) lse_out[row] = lse;
    const int64_t t = target[row];
    if (t != pad) {
      const float zt = (float)zr[t];
      const float eps_i = eps / (V - 1);
      const float nl = lse - zt;
      const float smooth = V * lse - sum;
      nll += nl;
      loss += (1.f - eps - eps_i) * nl + eps_i * smooth;
    }
  }
  if (lane == 0) { red[0][w] = loss; red[1][w] = nll; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[gridDim.x + blockIdx.x] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// the nb block partials summed in a fixed order (one wave): acc[0..1] += {loss, nll} and / or
// call_out[0..1] = {loss, nll} (either may be null)
__global__ void __launch_bounds__(64) ls_xent_sum_kernel(const float* __restrict__ part, int nb,
                                                         float* __restrict__ acc, float* __restrict__ call_out) {
  float l = 0.f, n = 0.f;
  for (int i = threadIdx.x; i < nb; i += 64) { l += part[i]; n += part[nb + i]; }
  l = wave_sum(l);
  n = wave_sum(n);
  if (threadIdx.x == 0) {
    if (acc) { acc[0] += l; acc[1] += n; }
    if (call_out) { call_out[0] = l; call_out[1] = n; }
  }
}

template <int CPL>
__global__ void __launch_bounds__(256) ls_xent_bwd_kernel(const h16* __restrict__ z, long ld,
                                                          const int64_t* __restrict__ target, long rows,
                                                          int V, float eps, int pad, const float* __restrict__ lse,
                                                          const float* __restrict__ grad, h16* __restrict__ dz) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t t = target[row];
  const float g = grad[0];
  const float eps_i = eps / (V - 1);
  const float a = (t == pad) ? 0.f : g * (1.f - eps - eps_i);
  const float bsm = (t == pad) ? 0.f : g * eps_i;
  const float L = lse[row];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + c * 64) * 4;
    if (j0 < V) {
      h16x4 zv = *reinterpret_cast<const h16x4*>(z + row * ld + j0);
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = j0 + e;
        const float p = __expf((float)zv[e] - L);
        o[e] = (j < V) ? a * (p - (j == t ? 1.f : 0.f)) + bsm * (V * p - 1.f) : 0.f;
      }
      *reinterpret_cast<h16x4*>(dz + row * ld + j0) = h16x4{(h16)o[0], (h16)o[1], (h16)o[2], (h16)o[3]};
    }
  }
  // pad columns [V, ld) are written as zeros: the tied-embedding dgrad reduces over a K padded to
  // whole 64-wide k-tiles
  for (long j = V + lane; j < ld; j += 64) dz[row * ld + j] = (h16)0.f;
}

__global__ void grad_sqnorm_kernel(const h16* __restrict__ g, long n, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const long n8 = n / 8, S = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  // four 16-B loads in flight per thread before the first add (one at a time left the sweep
  // latency-bound); the per-thread summation order is the strided loop's
  for (; i + 3 * S < n8; i += 4 * S) {
    h16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const h16x8*>(g + (i + u * S) * 8);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float x = (float)v[u][e]; s += x * x; }
  }
  for (; i < n8; i += S) {
    h16x8 v = *reinterpret_cast<const h16x8*>(g + i * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float x = (float)v[e]; s += x * x; }
  }
  for (long i = n8 * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = (float)g[i];
    s += x * x;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// ost layout (device fp32 optimizer state, see include/mms2ut.h MMS_OST_*)
__global__ void grad_norm_finalize_kernel(const float* __restrict__ part, int nparts, float* ost,
                                          const float* __restrict__ sample_size) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 64) s += part[i];
  s = wave_sum_d(s);
  if (threadIdx.x == 0) {
    // FP16Optimizer: multiply factor = 1/loss_scale * 1/sample_size (grads all-reduced as a SUM)
    const float ss = sample_size ? fmaxf(sample_size[0], 1.f) : 1.f;
    const float mult = 1.f / (ost[MMS_OST_LOSS_SCALE] * ss);
    const float norm = (float)sqrt(s) * mult;
    ost[MMS_OST_MULT] = mult;
    ost[MMS_OST_GNORM] = norm;
    ost[MMS_OST_OVERFLOW] = (isfinite(norm) && isfinite((float)s)) ? 0.f : 1.f;
  }
}

// one thread: Adam step count / step size / clip coefficient and fairseq DynamicLossScaler
__global__ void optim_prepare_kernel(float* ost, float lr_peak, float warmup_init_lr, float warmup_updates,
                                     float b1, float b2, float clip, float scale_window, float min_scale) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  // FATAL is sticky: fairseq raises (FloatingPointError) at the first fatal step, so no later step
  // may update anything; every rank holds the same state vector and stops at the same step
  if (ost[MMS_OST_FATAL] != 0.f) return;
  if (ost[MMS_OST_INCONSISTENT] != 0.f) {
    // fairseq Trainer._check_grad_norms raised: no update, the run is dead (FATAL for the host)
    ost[MMS_OST_FATAL] = 1.f;
    return;
  }
  const bool overflow = ost[MMS_OST_OVERFLOW] != 0.f;
  float it = ost[MMS_OST_ITER];
  if (overflow) {
    // check_overflow (tolerance 0): decrease, remember, skip the update
    const float prev = ost[MMS_OST_LOSS_SCALE];
    ost[MMS_OST_LAST_OVERFLOW] = it;
    float ns = prev / 2.f;
    ost[MMS_OST_LAST_RESCALE] = it;
    if (ns <= min_scale) { ns = prev; ost[MMS_OST_FATAL] = 1.f; }
    ost[MMS_OST_LOSS_SCALE] = ns;
    ost[MMS_OST_ITER] = it + 1.f;
    return;
  }
  // fairseq inverse_sqrt at num_updates = completed (non-skipped) updates: the schedule only
  // advances on a real step (Trainer.train_step skips set_num_updates on overflow)
  const float nu = ost[MMS_OST_STEP];
  float lr;
  if (warmup_updates > 0.f && nu < warmup_updates)
    lr = warmup_init_lr + nu * ((lr_peak - warmup_init_lr) / warmup_updates);
  else
    lr = lr_peak * sqrtf(fmaxf(warmup_updates, 1.f)) * rsqrtf(fmaxf(nu, 1.f));
  ost[MMS_OST_LR] = lr;
  const float step = nu + 1.f;
  ost[MMS_OST_STEP] = step;
  const double bc1 = 1.0 - pow((double)b1, (double)step), bc2 = 1.0 - pow((double)b2, (double)step);
  ost[MMS_OST_STEP_SIZE] = (float)(lr * sqrt(bc2) / bc1);
  // FP16Optimizer.clip_grad_norm with a scaler: multiply_factor *= max_norm / norm when norm > max_norm
  const float gn = ost[MMS_OST_GNORM];
  ost[MMS_OST_CLIP_COEF] = (clip > 0.f && gn > clip) ? clip / gn : 1.f;
  // scaler.update(): grow every scale_window clean iterations
  const float since = it - ost[MMS_OST_LAST_OVERFLOW];
  if (fmodf(since, scale_window) == 0.f) {
    ost[MMS_OST_LOSS_SCALE] *= 2.f;
    ost[MMS_OST_LAST_RESCALE] = it;
  }
  ost[MMS_OST_ITER] = it + 1.f;
}

// One thread per 8 parameters: 16-B fp16 param / grad accesses, 2 x 16-B fp32 master / m / v
// accesses (the flat buffers are 8-element aligned per tensor, so every optimizer chunk starts on
// a 16-B boundary); a scalar tail covers n % 8.  Per-element arithmetic is the scalar update's.
MMS_DEV void adam_elem(float g, float& p, float& mi, float& vi, float lr, float step_size, float b1, float b2,
                       float eps, float wd) {
  if (wd != 0.f) p -= wd * lr * p;
  mi = b1 * mi + (1.f - b1) * g;
  vi = b2 * vi + (1.f - b2) * g * g;
  p -= step_size * mi / (sqrtf(vi) + eps);
}

__global__ void __launch_bounds__(256) adam_kernel(h16* __restrict__ param, const h16* __restrict__ grad,
                                                   float* __restrict__ master, float* __restrict__ m,
                                                   float* __restrict__ v, long n, const float* __restrict__ ost,
                                                   float b1, float b2, float eps, float wd) {
  // overflow: skip (FP16Optimizer OverflowError path); inconsistent grads across ranks: no update
  if (ost[MMS_OST_OVERFLOW] != 0.f || ost[MMS_OST_INCONSISTENT] != 0.f || ost[MMS_OST_FATAL] != 0.f) return;
  const float lr = ost[MMS_OST_LR];
  const float mult = ost[MMS_OST_MULT] * ost[MMS_OST_CLIP_COEF];
  const float step_size = ost[MMS_OST_STEP_SIZE];
  const long n8 = n / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const h16x8 gv = *reinterpret_cast<const h16x8*>(grad + 8 * i);
    f32x4 p[2], mv[2], vv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      p[h] = *reinterpret_cast<const f32x4*>(master + 8 * i + 4 * h);
      mv[h] = *reinterpret_cast<const f32x4*>(m + 8 * i + 4 * h);
      vv[h] = *reinterpret_cast<const f32x4*>(v + 8 * i + 4 * h);
    }
    h16x8 out;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float pe = p[e >> 2][e & 3], me = mv[e >> 2][e & 3], ve = vv[e >> 2][e & 3];
      adam_elem((float)gv[e] * mult, pe, me, ve, lr, step_size, b1, b2, eps, wd);
      p[e >> 2][e & 3] = pe;
      mv[e >> 2][e & 3] = me;
      vv[e >> 2][e & 3] = ve;
      out[e] = (h16)pe;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      *reinterpret_cast<f32x4*>(master + 8 * i + 4 * h) = p[h];
      *reinterpret_cast<f32x4*>(m + 8 * i + 4 * h) = mv[h];
      *reinterpret_cast<f32x4*>(v + 8 * i + 4 * h) = vv[h];
    }
    *reinterpret_cast<h16x8*>(param + 8 * i) = out;
  }
  for (long i = 8 * n8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float p = master[i], mi = m[i], vi = v[i];
    adam_elem((float)grad[i] * mult, p, mi, vi, lr, step_size, b1, b2, eps, wd);
    m[i] = mi;
    v[i] = vi;
    master[i] = p;
    param[i] = (h16)p;
  }
}

// fairseq Trainer._check_grad_norms, on device: every rank writes its grad norm into its slot of
// a zeroed [world] buffer (stage 0), the buffer is SUM-all-reduced, and stage 1 flags the step
// when the norms are finite and differ: max|n_r - n_0| / (n_0 + 1e-6) >= 1e-6.
__global__ void grad_norm_check_kernel(float* buf, int world, int rank, float* ost, int stage) {
  const int i = threadIdx.x;
  if (stage == 0) {
    for (int r = i; r < world; r += blockDim.x) buf[r] = (r == rank) ? ost[MMS_OST_GNORM] : 0.f;
    return;
  }
  if (i != 0) return;
  bool finite = true;
  float dmax = 0.f;
  for (int r = 0; r < world; ++r) {
    finite = finite && isfinite(buf[r]);
    dmax = fmaxf(dmax, fabsf(buf[r] - buf[0]));
  }
  // sticky: once a step was inconsistent the flag stays set (the host reads it at its log cadence)
  if (finite && dmax / (buf[0] + 1e-6f) >= 1e-6f) ost[MMS_OST_INCONSISTENT] = 1.f;
}

// x *= alpha (fp16, in place): DDP's pre-division of a gradient bucket by the world size
__global__ void scale_f16_kernel(h16* __restrict__ x, long n8, float alpha) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    h16x8 v = *reinterpret_cast<const h16x8*>(x + i * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (h16)((float)v[e] * alpha);
    *reinterpret_cast<h16x8*>(x + i * 8) = v;
  }
}

// acc (fp32) += x (fp16): gradient accumulation across --update-freq micro-batches
__global__ void accum_f16_f32_kernel(float* __restrict__ acc, const h16* __restrict__ x, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const h16x8 v = *reinterpret_cast<const h16x8*>(x + i * 8);
    f32x4 a = *reinterpret_cast<const f32x4*>(acc + i * 8);
    f32x4 b = *reinterpret_cast<const f32x4*>(acc + i * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { a[e] += (float)v[e]; b[e] += (float)v[e + 4]; }
    *reinterpret_cast<f32x4*>(acc + i * 8) = a;
    *reinterpret_cast<f32x4*>(acc + i * 8 + 4) = b;
  }
}

template <typename F>
int pick_cpl_v(int V, F&& f) {
  const int cpl = (V + 255) / 256;
  if (cpl <= 1) return f(std::integral_constant<int, 1>{});
  if (cpl <= 2) return f(std::integral_constant<int, 2>{});
  if (cpl <= 4) return f(std::integral_constant<int, 4>{});
  if (cpl <= 8) return f(std::integral_constant<int, 8>{});
  if (cpl <= 16) return f(std::integral_constant<int, 16>{});
  mms::set_error("ls_xent: vocabulary too large (%d)", V);
  return 1;
}

}  // namespace

extern "C" int mms2ut_ls_xent_fwd_log(const h16* logits, int64_t ld, const int64_t* target, int64_t rows, int V,
                                      float eps, int pad_idx, float* lse, float* part, float* acc, float* call_out,
                                      hipStream_t s) {
  MMS_REQUIRE(ld % 4 == 0 && ld >= V, "ls_xent: ld must be a multiple of 4 and >= V");
  MMS_REQUIRE(part && (acc || call_out), "ls_xent: null partials / loss");
  if (rows == 0) {
    if (call_out) {
      const float z[2] = {0.f, 0.f};
      return mms2ut_set_f32(call_out, 2, z, s);
    }
    return 0;
  }
  const int nb = (int)std::min<long>((rows + 3) / 4, MMS_LS_XENT_PARTS);
  const int rc = pick_cpl_v(V, [&](auto C) {
    hipLaunchKernelGGL((ls_xent_fwd_kernel<decltype(C)::value>), dim3(nb), dim3(256), 0, s,
                       logits, (long)ld, target, (long)rows, V, eps, pad_idx, lse, part);
    return mms::check_launch("ls_xent_fwd");
  });
  if (rc) return rc;
  hipLaunchKernelGGL(ls_xent_sum_kernel, dim3(1), dim3(64), 0, s, part, nb, acc, call_out);
  return mms::check_launch("ls_xent_sum");
}

extern "C" int mms2ut_ls_xent_fwd(const h16* logits, int64_t ld, const int64_t* target, int64_t rows, int V,
                                  float eps, int pad_idx, float* lse, float* part, float* loss_out,
                                  hipStream_t s) {
  MMS_REQUIRE(loss_out, "ls_xent: null loss");
  return mms2ut_ls_xent_fwd_log(logits, ld, target, rows, V, eps, pad_idx, lse, part, loss_out, nullptr, s);
}

extern "C" int mms2ut_ls_xent_bwd(const h16* logits, int64_t ld, const int64_t* target, int64_t rows, int V,
                                  float eps, int pad_idx, const float* lse, const float* grad, h16* dlogits,
                                  hipStream_t s) {
  MMS_REQUIRE(ld % 4 == 0 && ld >= V, "ls_xent_bwd: ld must be a multiple of 4 and >= V");
  if (rows == 0) return 0;
  return pick_cpl_v(V, [&](auto C) {
    hipLaunchKernelGGL((ls_xent_bwd_kernel<decltype(C)::value>), dim3((rows + 3) / 4), dim3(256), 0, s,
                       logits, (long)ld, target, (long)rows, V, eps, pad_idx, lse, grad, dlogits);
    return mms::check_launch("ls_xent_bwd");
  });
}

extern "C" int mms2ut_grad_sqnorm(const h16* grad, int64_t n, float* part, int nparts, hipStream_t s) {
  MMS_REQUIRE(((uintptr_t)grad & 15) == 0, "grad_sqnorm: grad must be 16-byte aligned");
  MMS_REQUIRE(nparts > 0 && nparts <= 65535, "grad_sqnorm: bad nparts");
  hipLaunchKernelGGL(grad_sqnorm_kernel, dim3(nparts), dim3(256), 0, s, grad, (long)n, part);
  return mms::check_launch("grad_sqnorm");
}

extern "C" int mms2ut_grad_norm_finalize(const float* part, int nparts, float* ost, const float* sample_size,
                                         hipStream_t s) {
  hipLaunchKernelGGL(grad_norm_finalize_kernel, dim3(1), dim3(64), 0, s, part, nparts, ost, sample_size);
  return mms::check_launch("grad_norm_finalize");
}

extern "C" int mms2ut_optim_prepare(float* ost, float lr, float warmup_init_lr, float warmup_updates,
                                    float beta1, float beta2, float clip_norm, float scale_window,
                                    float min_loss_scale, hipStream_t s) {
  MMS_REQUIRE(scale_window >= 1.f, "optim_prepare: scale_window must be >= 1");
  MMS_REQUIRE(warmup_updates >= 0.f, "optim_prepare: warmup_updates must be >= 0");
  hipLaunchKernelGGL(optim_prepare_kernel, dim3(1), dim3(64), 0, s, ost, lr, warmup_init_lr, warmup_updates,
                     beta1, beta2, clip_norm, scale_window, min_loss_scale);
  return mms::check_launch("optim_prepare");
}

extern "C" int mms2ut_adam_fp16_master(h16* param, const h16* grad, float* master, float* exp_avg,
                                       float* exp_avg_sq, int64_t n, const float* ost, float beta1,
                                       float beta2, float eps, float weight_decay, hipStream_t s) {
  if (n == 0) return 0;
  MMS_REQUIRE(((uintptr_t)param & 15) == 0 && ((uintptr_t)grad & 15) == 0 && ((uintptr_t)master & 15) == 0 &&
                  ((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0,
              "adam: buffers must be 16-B aligned");
  long g = (n / 8 + 255) / 256;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(adam_kernel, dim3((int)g), dim3(256), 0, s, param, grad, master, exp_avg, exp_avg_sq,
                     (long)n, ost, beta1, beta2, eps, weight_decay);
  return mms::check_launch("adam");
}

extern "C" int mms2ut_grad_norm_check(float* buf, int world, int rank, float* ost, int stage, hipStream_t s) {
  MMS_REQUIRE(world >= 1 && rank >= 0 && rank < world && (stage == 0 || stage == 1),
              "grad_norm_check: world=%d rank=%d stage=%d", world, rank, stage);
  hipLaunchKernelGGL(grad_norm_check_kernel, dim3(1), dim3(64), 0, s, buf, world, rank, ost, stage);
  return mms::check_launch("grad_norm_check");
}

extern "C" int mms2ut_scale_f16(h16* x, int64_t n, float alpha, hipStream_t s) {
  MMS_REQUIRE(n % 8 == 0 && ((uintptr_t)x & 15) == 0, "scale_f16: n %% 8 == 0 and 16-B alignment");
  if (n == 0) return 0;
  const long n8 = n / 8;
  const long nb = std::min<long>((n8 + 255) / 256, 4096);
  hipLaunchKernelGGL(scale_f16_kernel, dim3(nb), dim3(256), 0, s, x, n8, alpha);
  return mms::check_launch("scale_f16");
}

struct F32x8 { float v[8]; };
__global__ void set_f32_kernel(float* __restrict__ dst, int n, F32x8 vals) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = vals.v[threadIdx.x];
}

extern "C" int mms2ut_set_f32(float* dst, int n, const float* vals, hipStream_t s) {
  MMS_REQUIRE(dst && vals && n >= 0 && n <= 8, "set_f32: 0 <= n <= 8 values (got %d)", n);
  if (n == 0) return 0;
  F32x8 v{};
  for (int i = 0; i < n; ++i) v.v[i] = vals[i];
  hipLaunchKernelGGL(set_f32_kernel, dim3(1), dim3(64), 0, s, dst, n, v);
  return mms::check_launch("set_f32");
}

extern "C" int mms2ut_accum_f16_f32(float* acc, const h16* x, int64_t n, hipStream_t s) {
  MMS_REQUIRE(n % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)acc & 15) == 0,
              "accum_f16_f32: n %% 8 == 0 and 16-B alignment");
  if (n == 0) return 0;
  const long n8 = n / 8;
  const long nb = std::min<long>((n8 + 255) / 256, 4096);
  hipLaunchKernelGGL(accum_f16_f32_kernel, dim3(nb), dim3(256), 0, s, acc, x, n8);
  return mms::check_launch("accum_f16_f32");
}
