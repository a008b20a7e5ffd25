// Kaldi-compatible 80-bin log-mel filterbank (torchaudio.compliance.kaldi.fbank defaults, the
// path the reference's get_fbank takes: mm_s2ut/data/audio_utils.py:326-349) + utterance CMVN +
// zero-padded fp16 collation.  One wave per 25 ms frame: DC removal and pre-emphasis through
// LDS, povey window, 512-point radix-2 complex FFT in LDS (twiddles from a table), power
// spectrum, sparse triangular mel filters, log(max(x, FLT_EPSILON)).  HBM-bound: 640 B of wave
// read (400 samples, hop 160 -> 4 B/sample amortised) + 320 B of features written per frame.
#include <algorithm>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

constexpr int WIN = 400, SHIFT = 160, NFFT = 512, NBIN = 257;

struct FbankConst {
  float window[WIN];
  float tw_re[NFFT / 2], tw_im[NFFT / 2];
};

__constant__ FbankConst c_fb;
static bool g_fb_init = false;

MMS_DEV int bitrev9(int x) { return (int)(__builtin_bitreverse32((unsigned)x) >> 23); }

__global__ void __launch_bounds__(256) fbank_kernel(const float* __restrict__ wave, const int64_t* __restrict__ wave_off,
                                                    const int* __restrict__ frame_off, int B, int total,
                                                    const float* __restrict__ banks,
                                                    const int* __restrict__ mel_range, int nbins,
                                                    float* __restrict__ feats) {
  __shared__ float s_re[4][NFFT], s_im[4][NFFT], s_x[4][WIN + 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int f = blockIdx.x * 4 + w;
  if (f >= total) return;
  // utterance of this frame (binary search over frame_off)
  int lo = 0, hi = B;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (frame_off[mid] <= f) lo = mid; else hi = mid;
  }
  const int b = lo;
  const int t = f - frame_off[b];
  const float* src = wave + wave_off[b] + (long)t * SHIFT;
  float* X = s_x[w];
  float* re = s_re[w];
  float* im = s_im[w];
  float sum = 0.f;
  for (int j = lane; j < WIN; j += 64) { const float v = src[j]; X[j] = v; sum += v; }
  const float mean = wave_sum(sum) / WIN;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // pre-emphasis (replicate-pad at j=0), window, scatter into bit-reversed order
  for (int j = lane; j < NFFT; j += 64) {
    float v = 0.f;
    if (j < WIN) {
      const float xj = X[j] - mean;
      const float xp = (j > 0 ? X[j - 1] : X[0]) - mean;
      v = (xj - 0.97f * xp) * c_fb.window[j];
    }
    const int r = bitrev9(j);
    re[r] = v;
    im[r] = 0.f;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // iterative radix-2 DIT, 9 stages, 256 butterflies per stage (4 per lane)
  for (int s = 1; s <= 9; ++s) {
    const int half = 1 << (s - 1);
    const int tstride = NFFT >> s;  // twiddle index stride
    float ar[4], ai[4], br[4], bi[4];
    int i0s[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int bfly = lane + q * 64;
      const int grp = bfly >> (s - 1), k = bfly & (half - 1);
      const int i0 = grp * (half << 1) + k;
      i0s[q] = i0;
      const float wr = c_fb.tw_re[k * tstride], wi = c_fb.tw_im[k * tstride];
      const float xr = re[i0 + half], xi = im[i0 + half];
      const float tr = wr * xr - wi * xi, ti = wr * xi + wi * xr;
      const float ur = re[i0], ui = im[i0];
      ar[q] = ur + tr; ai[q] = ui + ti; br[q] = ur - tr; bi[q] = ui - ti;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      re[i0s[q]] = ar[q]; im[i0s[q]] = ai[q];
      re[i0s[q] + half] = br[q]; im[i0s[q] + half] = bi[q];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  // power spectrum into X (reuse), bins 0..256
  for (int k = lane; k < NBIN; k += 64) X[k] = re[k] * re[k] + im[k] * im[k];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const float flt_eps = 1.1920928955078125e-07f;
  for (int m = lane; m < nbins; m += 64) {
    const float* bk = banks + (long)m * NBIN;
    float acc = 0.f;
    const int k0 = mel_range[2 * m], k1 = mel_range[2 * m + 1];  // triangle support only
    for (int k = k0; k < k1; ++k) acc += bk[k] * X[k];
    feats[(long)f * nbins + m] = __logf(fmaxf(acc, flt_eps));
  }
}

__global__ void fbank_frames_kernel(const int64_t* wave_off, int B, int* n_frames) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long n = wave_off[b + 1] - wave_off[b];
  n_frames[b] = n < WIN ? 0 : (int)(1 + (n - WIN) / SHIFT);
}

constexpr int CMVN_CHUNK = 64;  // frames staged in LDS per round (64 x 256 x 4 B = 64 KiB max)

__global__ void __launch_bounds__(256) cmvn_collate_kernel(const float* __restrict__ feats, const int* __restrict__ frame_off,
                                    int B, int Tmax, int nbins, int cmvn, h16* __restrict__ out) {
  const int b = blockIdx.x;
  const int f0 = frame_off[b], T = frame_off[b + 1] - f0;
  __shared__ float s_mean[256], s_std[256];
  __shared__ __attribute__((aligned(16))) float s_chunk[CMVN_CHUNK * 256];
  // fairseq UtteranceCMVN in numpy float32: x.mean(0) and (x**2).sum(0) reduce over the outer
  // (time) axis sequentially, var = sq/T - mean^2 (float32 cancellation included, as the
  // reference), std = sqrt(max(var, 1e-10)), x = (x - mean) / std.
  // The sums keep that sequential order per column; the frames are staged CMVN_CHUNK at a time
  // into LDS by all threads with coalesced 16-B loads, so the per-column chains read LDS instead
  // of waiting out one global round trip per frame.
  float sm = 0.f, sq = 0.f;
  const int c = threadIdx.x;
  for (int t0 = 0; t0 < T; t0 += CMVN_CHUNK) {
    const int nt = min(CMVN_CHUNK, T - t0);
    const int nv = nt * nbins / 4;  // nbins % 4 == 0 (host check)
    const f32x4* src = reinterpret_cast<const f32x4*>(feats + (long)(f0 + t0) * nbins);
    for (int i = threadIdx.x; i < nv; i += blockDim.x) reinterpret_cast<f32x4*>(s_chunk)[i] = src[i];
    __syncthreads();
    if (c < nbins) {
      for (int t = 0; t < nt; ++t) {
        const float v = s_chunk[t * nbins + c];
        sm = __fadd_rn(sm, v);
        sq = __fadd_rn(sq, __fmul_rn(v, v));
      }
    }
    __syncthreads();
  }
  if (c < nbins) {
    const float mean = T > 0 ? __fdiv_rn(sm, (float)T) : 0.f;
    const float var = T > 0 ? __fsub_rn(__fdiv_rn(sq, (float)T), __fmul_rn(mean, mean)) : 1.f;
    s_mean[c] = cmvn ? mean : 0.f;
    s_std[c] = cmvn ? __fsqrt_rn(fmaxf(var, 1e-10f)) : 1.f;
  }
  __syncthreads();
  // normalise + collate, 4 consecutive bins per thread (16-B loads, 8-B stores)
  const long n = (long)Tmax * nbins;
  for (long i = 4 * threadIdx.x; i < n; i += 4 * blockDim.x) {
    const int t = (int)(i / nbins), c = (int)(i % nbins);
    h16x4 o = {(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
    if (t < T) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(feats + (long)(f0 + t) * nbins + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (h16)__fdiv_rn(__fsub_rn(v[e], s_mean[c + e]), s_std[c + e]);
    }
    *reinterpret_cast<h16x4*>(out + (long)b * n + i) = o;
  }
}

// fairseq SpecAugmentTransform (feature_transforms/specaugment.py), applied on the device to the
// collated fp16 features after CMVN: the host draws each utterance's masks (freq (f0, f) pairs
// then time (t0, t) pairs, width 0 = no mask); the mask value is the utterance's mean over its
// valid [T, nbins] region (the transform's default, mask_value=None) or the given constant.
// One block per utterance: a 4-wide reduction for the mean, then one pass that rewrites only the
// 4-bin groups touching a masked row or column.
__global__ void __launch_bounds__(256) specaugment_kernel(h16* __restrict__ x, const int* __restrict__ frame_off,
                                                          int Tmax, int nbins, const int* __restrict__ masks,
                                                          int n_freq, int n_time, int use_const, float mask_const) {
  const int b = blockIdx.x;
  const int T = frame_off[b + 1] - frame_off[b];
  const int* m = masks + (long)b * 2 * (n_freq + n_time);
  h16* xb = x + (long)b * Tmax * nbins;
  const long n = (long)T * nbins;
  __shared__ float s_red[256 / 64];
  __shared__ float s_val;
  if (!use_const) {
    float acc = 0.f;
    for (long i = 4 * threadIdx.x; i < n; i += 4 * blockDim.x) {
      const h16x4 v = *reinterpret_cast<const h16x4*>(xb + i);
      acc += ((float)v[0] + (float)v[1]) + ((float)v[2] + (float)v[3]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < (int)blockDim.x / 64; ++w) t += s_red[w];
      s_val = n > 0 ? t / (float)n : 0.f;
    }
    __syncthreads();
  }
  const h16 mv = (h16)(use_const ? mask_const : s_val);
  for (long i = 4 * threadIdx.x; i < n; i += 4 * blockDim.x) {
    const int t = (int)(i / nbins), c = (int)(i % nbins);
    bool row = false;
    for (int k = 0; k < n_time; ++k) row |= (t >= m[2 * (n_freq + k)]) & (t < m[2 * (n_freq + k)] + m[2 * (n_freq + k) + 1]);
    int hit = row ? 0xF : 0;
    for (int k = 0; k < n_freq && hit != 0xF; ++k) {
      const int f0 = m[2 * k], f1 = m[2 * k] + m[2 * k + 1];
#pragma unroll
      for (int e = 0; e < 4; ++e) hit |= ((c + e >= f0) & (c + e < f1)) << e;
    }
    if (hit) {
      h16x4 v = *reinterpret_cast<const h16x4*>(xb + i);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (hit & (1 << e)) v[e] = mv;
      *reinterpret_cast<h16x4*>(xb + i) = v;
    }
  }
}

int init_consts(hipStream_t s) {
  if (g_fb_init) return 0;
  FbankConst h;
  for (int i = 0; i < WIN; ++i) {
    const double hann = 0.5 - 0.5 * cos(2.0 * M_PI * i / (WIN - 1));
    h.window[i] = (float)pow(hann, 0.85);
  }
  for (int k = 0; k < NFFT / 2; ++k) {
    h.tw_re[k] = (float)cos(-2.0 * M_PI * k / NFFT);
    h.tw_im[k] = (float)sin(-2.0 * M_PI * k / NFFT);
  }
  if (hipMemcpyToSymbolAsync(HIP_SYMBOL(c_fb), &h, sizeof(h), 0, hipMemcpyHostToDevice, s) != hipSuccess) {
    mms::set_error("fbank: constant upload failed");
    return 1;
  }
  if (hipStreamSynchronize(s) != hipSuccess) {
    mms::set_error("fbank: constant upload sync failed");
    return 1;
  }
  g_fb_init = true;
  return 0;
}

}  // namespace

extern "C" int mms2ut_fbank_frames(const int64_t* wave_off, int B, int32_t* n_frames_out, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(fbank_frames_kernel, dim3((B + 255) / 256), dim3(256), 0, s, wave_off, B, n_frames_out);
  return mms::check_launch("fbank_frames");
}

extern "C" int mms2ut_fbank_f32(const float* wave, const int64_t* wave_off, const int32_t* frame_off, int B,
                                int total_frames, const float* mel_banks, const int32_t* mel_range, int nbins,
                                float* feats, hipStream_t s) {
  MMS_REQUIRE(nbins > 0 && nbins <= 256, "fbank: nbins must be in (0, 256]");
  MMS_REQUIRE(mel_range != nullptr, "fbank: mel_range required");
  if (init_consts(s)) return 1;
  if (total_frames == 0) return 0;
  hipLaunchKernelGGL(fbank_kernel, dim3((total_frames + 3) / 4), dim3(256), 0, s, wave, wave_off, frame_off, B,
                     total_frames, mel_banks, mel_range, nbins, feats);
  return mms::check_launch("fbank");
}

extern "C" int mms2ut_fbank_cmvn_collate(const float* feats, const int32_t* frame_off, int B, int Tmax,
                                         int nbins, int cmvn, h16* out, hipStream_t s) {
  MMS_REQUIRE(nbins <= 256 && nbins % 4 == 0, "cmvn: nbins must be a multiple of 4, <= 256");
  MMS_REQUIRE(((uintptr_t)feats & 15) == 0 && ((uintptr_t)out & 7) == 0, "cmvn: feats / out misaligned");
  if (B == 0) return 0;
  hipLaunchKernelGGL(cmvn_collate_kernel, dim3(B), dim3(256), 0, s, feats, frame_off, B, Tmax, nbins, cmvn, out);
  return mms::check_launch("fbank_cmvn_collate");
}

extern "C" int mms2ut_specaugment_f16(h16* x, const int32_t* frame_off, int B, int Tmax, int nbins,
                                      const int32_t* masks, int n_freq, int n_time, int use_const,
                                      float mask_value, hipStream_t s) {
  MMS_REQUIRE(nbins % 4 == 0 && ((uintptr_t)x & 7) == 0, "specaugment: nbins % 4 / alignment");
  MMS_REQUIRE(n_freq >= 0 && n_time >= 0, "specaugment: negative mask count");
  if (B == 0 || n_freq + n_time == 0) return 0;
  hipLaunchKernelGGL(specaugment_kernel, dim3(B), dim3(256), 0, s, x, frame_off, Tmax, nbins, masks, n_freq,
                     n_time, use_const, mask_value);
  return mms::check_launch("specaugment");
}
