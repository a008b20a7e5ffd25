// Kaldi-compatible 80-bin log-mel filterbank (torchaudio.compliance.kaldi.fbank defaults, the
// path the reference's get_fbank takes: mm_s2ut/data/audio_utils.py:326-349) + utterance CMVN +
// zero-padded fp16 collation.
//
// fbank_kernel: four frames per wave (16 lanes each), 4 waves per block, a persistent grid (frame
// quads dealt to the waves round-robin), so the per-block LDS tables are built once per block.  DC
// removal, pre-emphasis and the povey window in registers, then the 512-point real FFT as a
// 256-point complex FFT of the even/odd sample pairs (z[n] = x[2n] + i x[2n+1]) done four-step
// (16 x 16: register DFTs, one LDS transpose) and the standard split X[k] = E[k] + W^k O[k]; power
// spectrum, triangular mel filters from a compact per-block LDS copy of their nonzero weights,
// log(max(x, FLT_EPSILON)).
// HBM-bound: 640 B of wave read (400 samples, hop 160 -> 4 B/sample amortised) + 4 * nbins B of
// features written per frame.
#include <algorithm>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

constexpr int WIN = 400, SHIFT = 160, NFFT = 512, NBIN = 257;
constexpr int NC = 256;                        // complex FFT points (the real 512-point FFT's half)
constexpr int FB_WAVES = 4;                    // waves per block
constexpr int MELW_MAX = 1024;                 // nonzero mel weights staged per block (80 bins: ~510)
constexpr int FB_MAXB = 256;                   // utterances whose frame / sample offsets are staged in LDS

struct FbankConst {
  float window[WIN];
  float tw_re[NFFT / 2], tw_im[NFFT / 2];      // exp(-2 pi i k / 512), k < 256
};

__constant__ FbankConst c_fb;
static bool g_fb_init = false;

// base-4 digit reversal of an 8-bit index (256 = 4^4)
MMS_DEV int rev4(int x) { return ((x & 3) << 6) | ((x & 12) << 2) | ((x & 48) >> 2) | ((x & 192) >> 6); }

// Four frames per wave, 16 lanes per frame.  The 256-point complex FFT runs as 16 x 16 (four-step):
// n = 16 n1 + n2, k = k1 + 16 k2.  Lane n2 holds z[16 n1 + n2] for all n1 in registers and does a
// 16-point DFT over n1 (radix 4 x 4, constant twiddles), multiplies by W256^(n2 k1), and the frame's
// 16 lanes swap rows and columns once through a padded LDS tile; lane k1 then does the 16-point DFT
// over n2 and holds Z[k1 + 16 k2].  One more LDS round trip pairs Z[k] with Z[256 - k] for the real
// split, a third hands the power spectrum to the mel sums (lane c: filters c, c + 16, ...).  Three
// LDS hand-offs per four frames instead of eight per frame, and no per-stage index arithmetic.
constexpr int FR_W = 4;                        // frames per wave
constexpr int TSTR = 17;                       // row stride (float2) of the transpose tile: conflict-free

struct FbankSmem {
  float2 tw[NFFT / 2];                         // exp(-2 pi i j / 512), j < 256
  float2 win2[NC];                             // (window[2m], window[2m + 1]); 0 past the 400 samples
  float melw[MELW_MAX];
  int mlo[256], mlen[256], moff[256], ntot;
  int foff[FB_MAXB + 1];
  long woff[FB_MAXB];
  float2 buf[FB_WAVES][FR_W][16 * TSTR];       // transpose tile, then Z, then the power spectrum
};

// exp(-2 pi i j / 512) for 0 <= j < 512 (W^(j+256) = -W^j)
MMS_DEV float2 tw512(const FbankSmem& S, int j) {
  const float2 t = S.tw[j & 255];
  return (j & 256) ? make_float2(-t.x, -t.y) : t;
}

// in-register 16-point forward DFT, A[k] = sum_n a[n] exp(-2 pi i nk / 16), as 4 x 4: n = 4p + q,
// k = r + 4s: four 4-point DFTs over p, twiddles W16^(qr), four 4-point DFTs over q
MMS_DEV void dft4(float& r0, float& i0, float& r1, float& i1, float& r2, float& i2, float& r3, float& i3) {
  const float s0r = r0 + r2, s0i = i0 + i2, d0r = r0 - r2, d0i = i0 - i2;
  const float s1r = r1 + r3, s1i = i1 + i3, d1r = r1 - r3, d1i = i1 - i3;
  r0 = s0r + s1r; i0 = s0i + s1i;            // y0 = a0 + a1 + a2 + a3
  r1 = d0r + d1i; i1 = d0i - d1r;            // y1 = a0 - i a1 - a2 + i a3
  r2 = s0r - s1r; i2 = s0i - s1i;            // y2 = a0 - a1 + a2 - a3
  r3 = d0r - d1i; i3 = d0i + d1r;            // y3 = a0 + i a1 - a2 - i a3
}

MMS_DEV void dft16(float (&re)[16], float (&im)[16]) {
  // W16^e = (cos(pi e / 8), -sin(pi e / 8)), e = q r <= 9
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508977f, R2 = 0.70710678118654752f;
  constexpr float WC[10] = {1.f, C1, R2, S1, 0.f, -S1, -R2, -C1, -1.f, -C1};
  constexpr float WS[10] = {0.f, -S1, -R2, -C1, -1.f, -C1, -R2, -S1, 0.f, S1};
#pragma unroll
  for (int q = 0; q < 4; ++q) dft4(re[q], im[q], re[4 + q], im[4 + q], re[8 + q], im[8 + q], re[12 + q], im[12 + q]);
  // now element (p = r, q) holds B[q][r] at index 4r + q
#pragma unroll
  for (int q = 1; q < 4; ++q)
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      const int e = q * r, i = 4 * r + q;
      const float xr = re[i] * WC[e] - im[i] * WS[e], xi = re[i] * WS[e] + im[i] * WC[e];
      re[i] = xr;
      im[i] = xi;
    }
  float orr[16], oi[16];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a[8] = {re[4 * r], im[4 * r], re[4 * r + 1], im[4 * r + 1], re[4 * r + 2], im[4 * r + 2], re[4 * r + 3], im[4 * r + 3]};
    dft4(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]);
#pragma unroll
    for (int s = 0; s < 4; ++s) { orr[r + 4 * s] = a[2 * s]; oi[r + 4 * s] = a[2 * s + 1]; }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) { re[k] = orr[k]; im[k] = oi[k]; }
}

// intra-wave LDS hand-off: this wave's LDS writes are complete (no wait on its global stores, so
// a frame's feature stores stay in flight under the next frames' work)
MMS_DEV void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// 3 waves per SIMD (168 VGPRs, a few spilled; the LDS allows 3 blocks per CU): 60 us against 70 us
// at the compiler's own 186 VGPRs / 2 waves (profiles/round4_fbank_v2_ab.txt)
__global__ void __launch_bounds__(64 * FB_WAVES, 3) fbank_kernel(const float* __restrict__ wave,
                                                              const int64_t* __restrict__ wave_off,
                                                              const int* __restrict__ frame_off, int B, int total,
                                                              const float* __restrict__ banks,
                                                              const int* __restrict__ mel_range, int nbins,
                                                              float* __restrict__ feats) {
  __shared__ FbankSmem S;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < NFFT / 2; i += blockDim.x) S.tw[i] = make_float2(c_fb.tw_re[i], c_fb.tw_im[i]);
  for (int m = tid; m < NC; m += blockDim.x)
    S.win2[m] = 2 * m + 1 < WIN ? make_float2(c_fb.window[2 * m], c_fb.window[2 * m + 1]) : make_float2(0.f, 0.f);
  for (int m = tid; m < nbins; m += blockDim.x) {
    const int lo = mel_range[2 * m], hi = mel_range[2 * m + 1];
    S.mlo[m] = lo;
    S.mlen[m] = hi - lo;
  }
  // utterance offsets in LDS: a frame's utterance is then found without a chain of dependent
  // global loads
  const bool lds_off = B <= FB_MAXB;
  if (lds_off) {
    for (int i = tid; i <= B; i += blockDim.x) S.foff[i] = frame_off[i];
    for (int i = tid; i < B; i += blockDim.x) S.woff[i] = wave_off[i];
  }
  __syncthreads();
  if (w == 0) {
    // exclusive prefix sum of the filter lengths (nbins <= 256: 4 per lane, then a wave scan)
    int len4[4], loc = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = 4 * lane + e;
      len4[e] = m < nbins ? S.mlen[m] : 0;
      loc += len4[e];
    }
    int inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    int run = inc - loc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = 4 * lane + e;
      if (m < nbins) S.moff[m] = run;
      run += len4[e];
    }
    if (lane == 63) S.ntot = inc;
  }
  __syncthreads();
  const int nw = S.ntot;   // <= 2 * 257: each FFT bin lies in at most two triangular filters
  for (int i = tid; i < nw && i < MELW_MAX; i += blockDim.x) {
    int a = 0, b = nbins;
    while (b - a > 1) {
      const int mid = (a + b) >> 1;
      if (S.moff[mid] <= i) a = mid; else b = mid;
    }
    S.melw[i] = banks[(long)a * NBIN + S.mlo[a] + (i - S.moff[a])];
  }
  __syncthreads();
  const int g = lane >> 4, c = lane & 15;
  float2* T = S.buf[w][g];
  float* P = reinterpret_cast<float*>(T);
  const float flt_eps = 1.1920928955078125e-07f;
  int utt = 0;   // utterance of the lane's last frame (frames only move forward)
  auto frame_src = [&](int f) {
    if (lds_off) {
      while (utt + 1 < B && S.foff[utt + 1] <= f) ++utt;
      return wave + S.woff[utt] + (long)(f - S.foff[utt]) * SHIFT;
    }
    int lo = 0, hi = B;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (frame_off[mid] <= f) lo = mid; else hi = mid;
    }
    return wave + wave_off[lo] + (long)(f - frame_off[lo]) * SHIFT;
  };
  // lane c of a frame holds samples 2m, 2m + 1 of m = 16 n1 + c, n1 < 13 (m < 200: the 400 samples)
  constexpr int NR = (WIN / 2 + 15) / 16;
  float xe[NR], xo[NR];
  auto load_frame = [&](int f) {
    if (f < total) {
      const float* src = frame_src(f);
#pragma unroll
      for (int n1 = 0; n1 < NR; ++n1) {
        const int m = 16 * n1 + c;
        const bool in = m < WIN / 2;
        xe[n1] = in ? src[2 * m] : 0.f;
        xo[n1] = in ? src[2 * m + 1] : 0.f;
      }
    } else {
#pragma unroll
      for (int n1 = 0; n1 < NR; ++n1) xe[n1] = xo[n1] = 0.f;
    }
  };
  // persistent: wave (block, w) takes frames 4 (w + FB_WAVES block) + g, then + 4 FB_WAVES gridDim.x
  const int fstep = FR_W * FB_WAVES * gridDim.x;
  int f = FR_W * (blockIdx.x * FB_WAVES + w) + g;
  load_frame(f);
  for (int f0 = FR_W * (blockIdx.x * FB_WAVES + w); f0 < total; f0 += fstep, f += fstep) {
    float sum = 0.f;
#pragma unroll
    for (int n1 = 0; n1 < NR; ++n1) sum += xe[n1] + xo[n1];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 16);
    const float mean = sum * (1.f / WIN);
    // DC removal, pre-emphasis (x[-1] = x[0]), window; x[2m - 1] is lane c - 1's odd sample (lane
    // 15's of the previous row for c = 0)
    float zr[16], zi[16];
#pragma unroll
    for (int n1 = 0; n1 < NR; ++n1) {
      const float r = __shfl(xo[n1], (c + 15) & 15, 16);
      const float prev_row = n1 ? __shfl(xo[n1 - 1], 15, 16) : xe[0];
      const float pe = c ? r : prev_row;
      const float2 wv = S.win2[16 * n1 + c];
      const float e = xe[n1] - mean, o = xo[n1] - mean;
      zr[n1] = (e - 0.97f * (pe - mean)) * wv.x;
      zi[n1] = (o - 0.97f * e) * wv.y;
    }
#pragma unroll
    for (int n1 = NR; n1 < 16; ++n1) zr[n1] = zi[n1] = 0.f;
    load_frame(f + fstep);   // the next frames' samples stream in under this one's transform
    // 16-point DFTs over n1, twiddle W256^(c k1) = W512^(2 c k1), transpose through LDS
    dft16(zr, zi);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) {
      float2 y = make_float2(zr[k1], zi[k1]);
      if (k1) {
        const float2 t = tw512(S, 2 * c * k1);
        y = make_float2(zr[k1] * t.x - zi[k1] * t.y, zr[k1] * t.y + zi[k1] * t.x);
      }
      T[k1 * TSTR + c] = y;
    }
    wave_sync();
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
      const float2 y = T[c * TSTR + n2];
      zr[n2] = y.x;
      zi[n2] = y.y;
    }
    dft16(zr, zi);   // lane c: Z[c + 16 k2] at k2
    float2* Z = T;
    // (the buffer is rewritten in place: compiler fences keep every read of one phase ahead of the
    // next phase's writes; the LDS itself serves one wave's accesses in order)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) Z[c + 16 * k2] = make_float2(zr[k2], zi[k2]);
    wave_sync();
    // real-FFT split: X[k] = E + W512^k O, E = (Z[k] + conj Z[256-k]) / 2, O = -i (Z[k] - conj Z[256-k]) / 2
    float pw[16];
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
      const int k = c + 16 * k2;
      const float2 zn = Z[(NC - k) & (NC - 1)];
      const float zkr = zr[k2], zki = zi[k2];
      const float er = 0.5f * (zkr + zn.x), ei = 0.5f * (zki - zn.y);
      const float orr = 0.5f * (zki + zn.y), oi = -0.5f * (zkr - zn.x);
      const float2 t = tw512(S, k);
      const float xr = er + (orr * t.x - oi * t.y), xi = ei + (orr * t.y + oi * t.x);
      pw[k2] = xr * xr + xi * xi;
    }
    // k = 256 (Nyquist): E = Re Z[0], O = Im Z[0], W512^256 = -1
    const float nyq = (zr[0] - zi[0]) * (zr[0] - zi[0]);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) P[c + 16 * k2] = pw[k2];
    if (c == 0) P[NC] = nyq;
    wave_sync();
    if (f < total) {
      for (int m = c; m < nbins; m += 16) {
        const float* wm = S.melw + S.moff[m];
        const float* pm = P + S.mlo[m];
        float acc = 0.f;
        for (int j = 0; j < S.mlen[m]; ++j) acc += wm[j] * pm[j];
        feats[(long)f * nbins + m] = __logf(fmaxf(acc, flt_eps));
      }
    }
    wave_sync();
  }
}

__global__ void fbank_frames_kernel(const int64_t* wave_off, int B, int* n_frames) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long n = wave_off[b + 1] - wave_off[b];
  n_frames[b] = n < WIN ? 0 : (int)(1 + (n - WIN) / SHIFT);
}

// fairseq UtteranceCMVN (numpy float32: mean over time, var = E[x^2] - mean^2,
// std = sqrt(max(var, 1e-10)), x = (x - mean) / std).  cmvn_partial_kernel: grid (B, MMS_CMVN_SPLIT),
// block (b, s) sums the s-th slice of utterance b's frames; thread t takes column t % nbins over
// the slice's rows r = t / nbins (mod the row groups), in fp64; the groups are combined in a fixed
// order -> part[b][s] = {sum[nbins], sumsq[nbins]}.  cmvn_fold_kernel folds the slices in order ->
// stats[b] = {mean[nbins], std[nbins]}.  Deterministic; fp64 leaves only the reference's own fp32
// cancellation error, which the parity test bounds.
__global__ void __launch_bounds__(256) cmvn_partial_kernel(const float* __restrict__ feats, const int* __restrict__ frame_off,
                                                           int nbins, double* __restrict__ part) {
  const int b = blockIdx.x, sl = blockIdx.y, ns = gridDim.y;
  const int f0 = frame_off[b], T = frame_off[b + 1] - f0;
  const int t0 = (int)((long)T * sl / ns), t1 = (int)((long)T * (sl + 1) / ns);
  const int groups = blockDim.x / nbins;          // >= 1 (nbins <= 256)
  const int c = threadIdx.x % nbins, g = threadIdx.x / nbins;
  __shared__ double s_sum[256], s_sq[256];
  double sm = 0.0, sq = 0.0;
  if (g < groups) {
    const float* col = feats + (long)f0 * nbins + c;
    for (int t = t0 + g; t < t1; t += groups) {
      const double v = col[(long)t * nbins];
      sm += v;
      sq += v * v;
    }
  }
  s_sum[threadIdx.x] = sm;
  s_sq[threadIdx.x] = sq;
  __syncthreads();
  if (threadIdx.x < nbins) {
    double a = 0.0, q = 0.0;
    for (int k = 0; k < groups; ++k) { a += s_sum[k * nbins + threadIdx.x]; q += s_sq[k * nbins + threadIdx.x]; }
    double* out = part + ((long)b * ns + sl) * 2 * nbins;
    out[threadIdx.x] = a;
    out[nbins + threadIdx.x] = q;
  }
}

__global__ void __launch_bounds__(256) cmvn_fold_kernel(const double* __restrict__ part, const int* __restrict__ frame_off,
                                                        int nbins, int ns, int cmvn, float* __restrict__ stats) {
  const int b = blockIdx.x, c = threadIdx.x;
  if (c >= nbins) return;
  const int T = frame_off[b + 1] - frame_off[b];
  double a = 0.0, q = 0.0;
  for (int sl = 0; sl < ns; ++sl) {
    const double* p = part + ((long)b * ns + sl) * 2 * nbins;
    a += p[c];
    q += p[nbins + c];
  }
  float mean = 0.f, sd = 1.f;
  if (cmvn && T > 0) {
    const double mu = a / T;
    mean = (float)mu;
    sd = (float)sqrt(fmax(q / T - mu * mu, 1e-10));
  }
  stats[(long)b * 2 * nbins + c] = mean;
  stats[(long)b * 2 * nbins + nbins + c] = sd;
}

// normalise + collate [B][Tmax][nbins] fp16 (zero rows past each utterance's length): a flat
// grid-stride pass, 4 consecutive bins per thread (16-B loads, 8-B stores)
__global__ void __launch_bounds__(256) cmvn_apply_kernel(const float* __restrict__ feats, const int* __restrict__ frame_off,
                                                         int B, int Tmax, int nbins, const float* __restrict__ stats,
                                                         h16* __restrict__ out) {
  const long per = (long)Tmax * nbins / 4, n4 = (long)B * per;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / per);
    const long e = (i - (long)b * per) * 4;
    const int t = (int)(e / nbins), c = (int)(e % nbins);
    const int f0 = frame_off[b], T = frame_off[b + 1] - f0;
    h16x4 o = {(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
    if (t < T) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(feats + (long)(f0 + t) * nbins + c);
      const float* st = stats + (long)b * 2 * nbins;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (h16)((v[k] - st[c + k]) / st[nbins + c + k]);
    }
    *reinterpret_cast<h16x4*>(out + (long)b * Tmax * nbins + e) = o;
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
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  // persistent: as many blocks as fit on a CU at once (LDS / VGPR bound), each building its tables once
  static int per_cu = 0;
  if (per_cu == 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fbank_kernel, 64 * FB_WAVES, 0) != hipSuccess ||
                      per_cu <= 0))
    per_cu = 4;
  // a block consumes FR_W * FB_WAVES frames per sweep: no more blocks than that covers
  const int grid = std::min((total_frames + FR_W * FB_WAVES - 1) / (FR_W * FB_WAVES), per_cu * ncu);
  hipLaunchKernelGGL(fbank_kernel, dim3(grid), dim3(64 * FB_WAVES), 0, s, wave, wave_off,
                     frame_off, B, total_frames, mel_banks, mel_range, nbins, feats);
  return mms::check_launch("fbank");
}

extern "C" int mms2ut_fbank_cmvn_collate(const float* feats, const int32_t* frame_off, int B, int Tmax,
                                         int nbins, int cmvn, float* stats, h16* out, hipStream_t s) {
  MMS_REQUIRE(nbins > 0 && nbins <= 256 && nbins % 4 == 0, "cmvn: nbins must be a multiple of 4, <= 256");
  MMS_REQUIRE(((uintptr_t)feats & 15) == 0 && ((uintptr_t)out & 7) == 0 && stats, "cmvn: feats / out misaligned");
  if (B == 0) return 0;
  // fp64 slice partials after the fp32 stats (8-B aligned): see include/mms2ut.h
  double* part = reinterpret_cast<double*>(stats + ((2L * B * nbins + 1) & ~1L));
  hipLaunchKernelGGL(cmvn_partial_kernel, dim3(B, MMS_CMVN_SPLIT), dim3(256), 0, s, feats, frame_off, nbins, part);
  if (int rc = mms::check_launch("cmvn_partial")) return rc;
  hipLaunchKernelGGL(cmvn_fold_kernel, dim3(B), dim3(nbins), 0, s, part, frame_off, nbins, MMS_CMVN_SPLIT, cmvn, stats);
  if (int rc = mms::check_launch("cmvn_fold")) return rc;
  const long n4 = (long)B * Tmax * nbins / 4;
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(cmvn_apply_kernel, dim3((unsigned)std::min<long>((n4 + 255) / 256, 4096)), dim3(256), 0, s,
                     feats, frame_off, B, Tmax, nbins, stats, out);
  return mms::check_launch("cmvn_apply");
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
