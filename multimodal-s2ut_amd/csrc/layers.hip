// Transformer layers as single C-ABI calls: one fairseq pre-LN TransformerEncoderLayer /
// TransformerDecoderLayer (encoder_normalize_before / decoder_normalize_before) forward, and its
// hand-written backward with the weight gradients on a second (side) stream.
//
// The host used to issue these launches one by one from Python (~15 us of interpreter + ctypes
// per launch on top of the HIP runtime's own ~4 us, ~750 launches per training step); here the
// whole per-layer sequence is enqueued from C++ in one call.  The kernels, their arguments, the
// dropout counters and the stream order are exactly those of the per-launch path, so results are
// bit-identical to it (tests/test_gpu_layers.py checks that against the oracle-pinned model).
//
// Memory: the library still never allocates.  The forward writes every tensor the backward needs
// (and the layer output) into a caller-owned arena whose layout mms2ut_layer_arena() returns;
// the backward writes its temporaries (and dx) into a caller-owned scratch block
// (mms2ut_layer_scratch()) that must stay alive until the side stream has been joined, because
// the weight-gradient GEMMs read from it; split-K workspaces (fixups on the main stream, and
// weight-gradient slabs when a shape rules out the grouped launch) are caller-owned per-stream
// buffers sized by mms2ut_layer_ws().
//
// Weight gradients: the layer's projections (QKV, out-proj, fc1, fc2, + the decoder's
// cross-attention q / out) are collected during the dgrad chain and issued as ONE grouped, unsplit
// launch (mms2ut_wgrad_group) on the side stream at the end of the layer's backward — no fp32
// split-K slabs, no reduction launches; it overlaps the next layer's dgrad chain.
#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "../../include/mms2ut.h"

namespace {

constexpr int64_t kAlign = 256;   // bytes: every arena / scratch tensor starts 256-B aligned

int64_t al(int64_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

// ---------------------------------------------------------------- arena / scratch layouts
struct Dims {
  bool dec;
  int64_t R, Rk, d, F, BHT, BHTk;
};

Dims dims_of(const mms2ut_layer* L) {
  Dims D;
  D.dec = L->kind == MMS_LAYER_DEC;
  D.R = (int64_t)L->B * L->T;
  D.Rk = (int64_t)L->B * L->Tk;
  D.d = L->d;
  D.F = L->F;
  D.BHT = (int64_t)L->B * L->H * L->T;
  D.BHTk = D.BHT;   // cross attention: one LSE / D row per query
  return D;
}

// forward arena slots (bytes per slot), in layout order
void arena_sizes(const Dims& D, int64_t* sz) {
  const int64_t h = 2, f = 4;
  for (int i = 0; i < MMS_LAYER_NSLOT; ++i) sz[i] = 0;
  sz[MMS_SLOT_M1] = sz[MMS_SLOT_R1] = D.R * f;
  sz[MMS_SLOT_H1] = D.R * D.d * h;
  sz[MMS_SLOT_QKV] = D.R * 3 * D.d * h;
  sz[MMS_SLOT_LSE_SA] = D.BHT * f;
  sz[MMS_SLOT_O] = D.R * D.d * h;
  sz[MMS_SLOT_XA] = D.R * D.d * h;
  if (D.dec) {
    sz[MMS_SLOT_M2] = sz[MMS_SLOT_R2] = D.R * f;
    sz[MMS_SLOT_H2] = D.R * D.d * h;
    sz[MMS_SLOT_Q] = D.R * D.d * h;
    sz[MMS_SLOT_LSE_CA] = D.BHTk * f;
    sz[MMS_SLOT_CO] = D.R * D.d * h;
    sz[MMS_SLOT_XB] = D.R * D.d * h;
  }
  sz[MMS_SLOT_M3] = sz[MMS_SLOT_R3] = D.R * f;
  sz[MMS_SLOT_H3] = D.R * D.d * h;
  sz[MMS_SLOT_F1] = D.R * D.F * h;
  sz[MMS_SLOT_OUT] = D.R * D.d * h;
}

int64_t layout(const int64_t* sz, int n, int64_t* off) {
  int64_t o = 0;
  for (int i = 0; i < n; ++i) {
    off[i] = sz[i] ? o : -1;
    o += al(sz[i]);
  }
  return o;
}

// backward scratch slots
enum {
  S_DX = 0, S_DXD, S_DYD, S_DF1, S_DH3, S_DX3, S_DY3B, S_DO2, S_DQ, S_DD_CA, S_DH2, S_DX2, S_DY2B,
  S_DO, S_DQKV, S_DD_SA, S_DH1, S_P3, S_P2, S_P1, S_BPART, S_N
};

int ln_parts(int64_t R, int D) { return mms2ut_layernorm_bwd_nparts(R, D); }

// the grouped weight-gradient launch takes N, K (= d, F) multiples of 8 and row extents a buffer
// descriptor covers; otherwise each weight gradient is its own split-K launch
bool group_ok(const Dims& D) {
  return D.d % 8 == 0 && D.F % 8 == 0 && D.R * 3 * D.d * 2 < (1LL << 31) && D.R * D.F * 2 < (1LL << 31);
}

void scratch_sizes(const Dims& D, float emit_p, int64_t* sz) {
  const int64_t h = 2, f = 4, Rd = D.R * D.d * h;
  for (int i = 0; i < S_N; ++i) sz[i] = 0;
  sz[S_DX] = Rd;
  sz[S_DXD] = emit_p > 0.f ? Rd : 0;
  sz[S_DYD] = Rd;
  sz[S_DF1] = D.R * D.F * h;
  sz[S_DH3] = Rd;
  sz[S_DY3B] = Rd;   // dropout(dx of the FFN LN) = the residual-branch gradient of the block below
  if (D.dec) {
    sz[S_DX3] = Rd;
    sz[S_DO2] = Rd;
    sz[S_DQ] = Rd;
    sz[S_DD_CA] = D.BHTk * f;
    sz[S_DH2] = Rd;
    sz[S_DY2B] = Rd;
  }
  sz[S_DX2] = Rd;
  sz[S_DO] = Rd;
  sz[S_DQKV] = D.R * 3 * D.d * h;
  sz[S_DD_SA] = D.BHT * f;
  sz[S_DH1] = Rd;
  const int64_t lp = (int64_t)ln_parts(D.R, (int)D.d) * 2 * D.d * f;
  sz[S_P3] = lp;
  sz[S_P2] = D.dec ? lp : 0;
  sz[S_P1] = lp;
  // colsum partials of the bias-gradient fallback (wgrads whose shapes the fused row sums skip)
  sz[S_BPART] = (int64_t)mms2ut_colsum_nparts(D.R) * std::max<int64_t>(3 * D.d, D.F) * f;
}

// ---------------------------------------------------------------- launch helpers
struct Ctx {
  hipStream_t main, side;
  float* main_ws;
  int64_t main_ws_floats;
  float* side_ws;
  int64_t side_ws_floats;
  float* bpart;   // scratch for the bias-gradient fallback partials
  // the layer's weight gradients, collected for one grouped launch (mms2ut_wgrad_group) at the end
  // of the layer's backward; grouped = every problem meets the grouped kernel's shape rules
  mms2ut_wgrad* group;
  int* ngroup;
  bool grouped;
};

int fixup_splits(int64_t M, int64_t N, int64_t K) {
  // kernels.py _fixup_splits: short-M fused-epilogue GEMMs split K until ~512 workgroups run
  if (N % 4 || K < 512) return 1;
  const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
  if (tiles >= 128) return 1;
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(512 / tiles, K / 256), 16));
}

int wgrad_splits(int64_t tiles, int64_t kred) {
  // kernels.py _splitk_for: the largest split whose tiles*s blocks fit one round of 512 slots
  int s = (int)std::max<int64_t>(1, std::min<int64_t>(16, 512 / std::max<int64_t>(tiles, 1)));
  while (s > 1 && kred / s < 256) --s;
  return s;
}

mms2ut_gemm_args gemm_args() {
  mms2ut_gemm_args a = {};
  a.batch = 1;
  a.bdiv = 1;
  a.splitk = 1;
  a.alpha = 1.f;
  return a;
}

// C[M, N] = epi(A[M, K] @ B[N, K]^T + bias): the forward / dgrad shape (both operands
// K-contiguous unless b_kc = 0), with the short-M split-K fixup of kernels.gemm
int gemm_nt(const Ctx& c, const mms2ut_half* A, int64_t lda, const mms2ut_half* B, int64_t ldb, int b_kc,
            mms2ut_half* C, int64_t ldc, int64_t M, int64_t N, int64_t K, int epi, const mms2ut_half* bias,
            const mms2ut_half* aux, int64_t ldaux, float p, uint64_t seed, uint64_t off, int64_t ld_rng) {
  mms2ut_gemm_args a = gemm_args();
  a.A = A; a.B = B; a.C = C;
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.a_kcontig = 1; a.b_kcontig = b_kc;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.epi = epi; a.bias = bias; a.aux = aux; a.ldaux = ldaux;
  a.dropout_p = p; a.seed = seed; a.offset = off; a.ld_rng = ld_rng;
  const int s = fixup_splits(M, N, K);
  if (s > 1) {
    MMS_REQUIRE(c.main_ws && c.main_ws_floats >= (int64_t)s * M * N, "layer: main workspace too small for a split-K fixup");
    a.splitk = s;
    a.splitk_ws = c.main_ws;
    a.splitk_ws_floats = c.main_ws_floats;
  }
  return mms2ut_gemm_f16(&a, c.main);
}

// y = x @ W^T + b (nn.Linear) on the main stream
int linear(const Ctx& c, const mms2ut_half* x, const mms2ut_half* W, const mms2ut_half* b, mms2ut_half* y,
           int64_t M, int64_t N, int64_t K, int epi = MMS_EPI_F16, const mms2ut_half* aux = nullptr,
           float p = 0.f, uint64_t seed = 0, uint64_t off = 0) {
  return gemm_nt(c, x, K, W, K, 1, y, N, M, N, K, epi, b, aux, aux ? N : 0, p, seed, off, N);
}

// dx[M, K] = dy[M, N] @ W[N, K]: through the W^T image when there is one (both operands
// K-contiguous), else transposed reads of W (kernels.linear_dgrad)
int dgrad(const Ctx& c, const mms2ut_half* dy, int64_t lddy, const mms2ut_half* W, const mms2ut_half* WT,
          mms2ut_half* dx, int64_t M, int64_t N, int64_t K, int epi = MMS_EPI_F16, const mms2ut_half* aux = nullptr,
          float p = 0.f) {
  if (WT) return gemm_nt(c, dy, lddy, WT, N, 1, dx, K, M, K, N, epi, nullptr, aux, aux ? K : 0, p, 0, 0, K);
  return gemm_nt(c, dy, lddy, W, K, 0, dx, K, M, K, N, epi, nullptr, aux, aux ? K : 0, p, 0, 0, K);
}

int fork(const Ctx& c) { return c.side == c.main ? 0 : mms2ut_stream_wait(c.side, c.main); }

// MMS2UT_WGRAD_SPLIT (A/B): issue a layer's FFN weight gradients as a separate grouped launch
int wgrad_split_mode() {
  static int m = -1;
  if (m < 0) {
    const char* e = getenv("MMS2UT_WGRAD_SPLIT");
    m = e ? atoi(e) : 0;
  }
  return m;
}

// A layer's grouped weight gradients are held back and launched from inside the NEXT layer's
// backward, at flush point MMS2UT_WGRAD_DEFER (default 5: behind that layer's self-attention
// backward; 0 = at the end of their own layer, as before round 6).  Launched at the end of their
// own layer, the ~430-tile group took the CUs ahead of the next layer's FFN dgrads (the fc1 dgrad ran
// 4-5x its serial time beside it); behind the attention backward it shares the CUs with the
// QKV dgrad and the LayerNorm / attention kernels of the layers below instead.  Same-box A/Bs
// (profiles/round6_wgrad_defer_ab.txt): 16.20-16.31 -> 15.90-15.98 ms (point 5), 16.03-16.09 (1),
// 16.34-16.44 (3), 16.40-16.42 (4); points 2 and 6 lose (17.1).  Host thread-local (the backward
// issues from one thread); flushed by mms2ut_wgrad_flush before the side stream is joined or a
// gradient ready point is reported (data-parallel hooks), so a bucket never misses a gradient.
struct PendingGroup {
  bool on = false;
  mms2ut_wgrad w[8];
  int n = 0;
  int64_t rows = 0;
  int blocks = 0;
  hipStream_t side = nullptr;
};
thread_local PendingGroup g_pend;
int wgrad_defer_mode() {
  static int m = -1;
  if (m < 0) {
    const char* e = getenv("MMS2UT_WGRAD_DEFER");
    m = e ? atoi(e) : 5;
  }
  return m;
}
int flush_pending(hipStream_t main) {
  if (!g_pend.on) return 0;
  g_pend.on = false;
  int rc = g_pend.side == main ? 0 : mms2ut_stream_wait(g_pend.side, main);
  if (rc) return rc;
  return mms2ut_wgrad_group(g_pend.w, g_pend.n, g_pend.rows, g_pend.blocks, g_pend.side);
}

// dW[N, K] = dy[M, N]^T @ x[M, K] and db[N] = colsum(dy), on the side stream (kernels.linear_wgrad):
// fp32 split-K slabs with the bias partials as A-row sums, one reduction launch
int wgrad(const Ctx& c, const mms2ut_half* dy, int64_t lddy, const mms2ut_half* x, int64_t ldx, mms2ut_half* dW,
          mms2ut_half* db, int64_t M, int64_t N, int64_t K) {
  if (c.grouped) {
    c.group[(*c.ngroup)++] = mms2ut_wgrad{dy, lddy, x, ldx, dW, db, (int)N, (int)K};
    return 0;
  }
  int rc = fork(c);
  if (rc) return rc;
  const int64_t tiles = ((N + 127) / 128) * ((K + 127) / 128);
  const int s = wgrad_splits(tiles, M);
  const bool fused_db = db && K % 64 == 0 && N % 4 == 0;
  const int64_t need = (int64_t)s * N * K + (db ? (int64_t)s * N : 0);
  MMS_REQUIRE(c.side_ws && c.side_ws_floats >= need, "layer: side workspace too small (%ld < %ld floats)",
              (long)c.side_ws_floats, (long)need);
  float* slabs = c.side_ws;
  float* rs = c.side_ws + (int64_t)s * N * K;
  mms2ut_gemm_args a = gemm_args();
  a.A = dy; a.B = x; a.C = slabs;
  a.M = (int)N; a.N = (int)K; a.K = (int)M;
  a.a_kcontig = 0; a.b_kcontig = 0;
  a.lda = lddy; a.ldb = ldx; a.ldc = K;
  a.epi = MMS_EPI_F32; a.splitk = s; a.sCsplit = N * K;
  if (fused_db) { a.rowsum = rs; a.ld_rowsum = N; }
  if ((rc = mms2ut_gemm_f16(&a, c.side))) return rc;
  if (fused_db) return mms2ut_splitk_reduce_bias(slabs, s, N * K, (int)N, (int)K, dW, K, rs, db, c.side);
  if ((rc = mms2ut_splitk_reduce(slabs, s, N * K, (int)N, (int)K, dW, K, 1, 1.f, c.side))) return rc;
  if (!db) return 0;
  // kernels.bias_grad: column partials of dy, then their sums
  const int np = mms2ut_colsum_nparts(M);
  if ((rc = mms2ut_colsum_f16(dy, M, (int)N, lddy, c.bpart, np, c.side))) return rc;
  return mms2ut_colsum_parts(c.bpart, np, (int)N, db, 0, c.side);
}

// LayerNorm backward (+ residual gradient dres, + dropout(dx) for the sublayer below when p > 0);
// the gamma | beta partial sums are reduced on the side stream
int ln_bwd(const Ctx& c, const mms2ut_half* dy, const mms2ut_half* x, const mms2ut_half* g, const float* mean,
           const float* rstd, const mms2ut_half* dres, mms2ut_half* dx, mms2ut_half* dxd, float p, uint64_t seed,
           uint64_t off, float* part, mms2ut_half* dgb, int64_t R, int D) {
  int rc = mms2ut_layernorm_bwd(dy, x, g, mean, rstd, dres, dx, part, R, D, p > 0.f ? dxd : nullptr, p, seed, off,
                                c.main);
  if (rc || (rc = fork(c))) return rc;
  return mms2ut_colsum_parts(part, ln_parts(R, D), 2 * D, dgb, 0, c.side);
}

mms2ut_attn_args attn(const mms2ut_half* q, int64_t ldq, const mms2ut_half* k, const mms2ut_half* v, int64_t ldkv,
                      mms2ut_half* o, int64_t ldo, int B, int H, int Tq, int Tk, int hd, const int32_t* klen, int causal,
                      float p, uint64_t seed, uint64_t off, float* lse) {
  mms2ut_attn_args a = {};
  a.q = q; a.k = k; a.v = v; a.o = o;
  a.ldq = ldq; a.ldk = ldkv; a.ldv = ldkv; a.ldo = ldo;
  a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.hd = hd;
  a.key_len = klen; a.causal = causal;
  a.scale = (float)pow((double)hd, -0.5);   // float(hd ** -0.5) as the per-launch path packs it
  a.p = p; a.seed = p > 0.f ? seed : 0; a.offset = p > 0.f ? off : 0;
  a.lse = lse;
  return a;
}

template <typename T>
T* at(void* base, const int64_t* off, int slot) {
  return off[slot] < 0 ? nullptr : reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off[slot]);
}

}  // namespace

extern "C" int mms2ut_layer_arena(const mms2ut_layer* L, int64_t* offsets, int64_t* bytes) {
  MMS_REQUIRE(L && bytes, "layer_arena: null");
  int64_t sz[MMS_LAYER_NSLOT], off[MMS_LAYER_NSLOT];
  arena_sizes(dims_of(L), sz);
  *bytes = layout(sz, MMS_LAYER_NSLOT, off);
  if (offsets) std::copy(off, off + MMS_LAYER_NSLOT, offsets);
  return 0;
}

extern "C" int mms2ut_layer_scratch(const mms2ut_layer* L, float emit_p, int64_t* dx_offsets, int64_t* bytes) {
  MMS_REQUIRE(L && bytes, "layer_scratch: null");
  int64_t sz[S_N], off[S_N];
  scratch_sizes(dims_of(L), emit_p, sz);
  *bytes = layout(sz, S_N, off);
  if (dx_offsets) { dx_offsets[0] = off[S_DX]; dx_offsets[1] = off[S_DXD]; }
  return 0;
}

extern "C" int mms2ut_layer_ws(const mms2ut_layer* L, int64_t* main_floats, int64_t* side_floats) {
  MMS_REQUIRE(L && main_floats && side_floats, "layer_ws: null");
  const Dims D = dims_of(L);
  int64_t mw = 0, sw = 0;
  auto fw = [&](int64_t M, int64_t N, int64_t K) {
    const int s = fixup_splits(M, N, K);
    if (s > 1) mw = std::max(mw, (int64_t)s * M * N);
  };
  auto ww = [&](int64_t M, int64_t N, int64_t K) {
    const int s = wgrad_splits(((N + 127) / 128) * ((K + 127) / 128), M);
    sw = std::max(sw, (int64_t)s * N * K + (int64_t)s * N);
  };
  const int64_t R = D.R, d = D.d, F = D.F;
  // forward / dgrad GEMMs (M, N, K)
  fw(R, 3 * d, d); fw(R, d, d); fw(R, F, d); fw(R, d, F);
  fw(R, d, 3 * d); fw(R, F, d); fw(R, d, F);
  // weight gradients (rows M, out N, in K): split-K slabs only without the grouped launch
  if (!group_ok(D)) {
    ww(R, 3 * d, d); ww(R, d, d); ww(R, F, d); ww(R, d, F);
    if (D.dec) ww(R, d, d);
  }
  if (D.dec) fw(R, d, d);
  *main_floats = mw;
  *side_floats = sw;
  return 0;
}

extern "C" int mms2ut_layer_fwd(const mms2ut_layer* L, float* main_ws, int64_t main_ws_floats, hipStream_t s) {
  MMS_REQUIRE(L && L->x && L->saved, "layer_fwd: null layer / input / arena");
  MMS_REQUIRE(L->kind == MMS_LAYER_ENC || L->kind == MMS_LAYER_DEC, "layer_fwd: kind %d", L->kind);
  MMS_REQUIRE(L->H > 0 && L->d % L->H == 0 && L->d % 8 == 0 && L->F % 8 == 0, "layer_fwd: d=%d H=%d F=%d", L->d, L->H, L->F);
  MMS_REQUIRE(L->kind != MMS_LAYER_DEC || (L->kv && L->ld_kv % 8 == 0), "layer_fwd: decoder needs kv (ld %% 8)");
  const Dims D = dims_of(L);
  int64_t sz[MMS_LAYER_NSLOT], off[MMS_LAYER_NSLOT];
  arena_sizes(D, sz);
  layout(sz, MMS_LAYER_NSLOT, off);
  void* A = L->saved;
  const Ctx c{s, s, main_ws, main_ws_floats, nullptr, 0, nullptr};
  const int64_t R = D.R, d = D.d, F = D.F;
  const int hd = L->d / L->H;
  int rc;
  // self-attention block: x -> LN -> q|k|v -> attention -> out_proj (+dropout +residual)
  mms2ut_half* h1 = at<mms2ut_half>(A, off, MMS_SLOT_H1);
  mms2ut_half* qkv = at<mms2ut_half>(A, off, MMS_SLOT_QKV);
  mms2ut_half* O = at<mms2ut_half>(A, off, MMS_SLOT_O);
  mms2ut_half* xa = at<mms2ut_half>(A, off, MMS_SLOT_XA);
  if ((rc = mms2ut_layernorm_fwd(L->x, L->ln1_g, L->ln1_b, h1, at<float>(A, off, MMS_SLOT_M1),
                                 at<float>(A, off, MMS_SLOT_R1), R, (int)d, L->eps, s))) return rc;
  if ((rc = linear(c, h1, L->w_qkv, L->b_qkv, qkv, R, 3 * d, d))) return rc;
  {
    mms2ut_attn_args a = attn(qkv, 3 * d, qkv + d, qkv + 2 * d, 3 * d, O, d, L->B, L->H, L->T, L->T, hd,
                              L->self_len, D.dec ? 1 : 0, L->p_attn, L->seed, L->off_sa_attn,
                              at<float>(A, off, MMS_SLOT_LSE_SA));
    if ((rc = mms2ut_mha_varlen_fwd(&a, s))) return rc;
  }
  if ((rc = linear(c, O, L->w_o, L->b_o, xa, R, d, d, MMS_EPI_DROP_RESID, L->x, L->p_drop, L->seed, L->off_sa_res)))
    return rc;
  const mms2ut_half* xf = xa;   // the FFN block's input
  if (D.dec) {
    // cross-attention block: LN -> q_proj -> attention over the precomputed encoder K | V -> out_proj
    mms2ut_half* h2 = at<mms2ut_half>(A, off, MMS_SLOT_H2);
    mms2ut_half* q = at<mms2ut_half>(A, off, MMS_SLOT_Q);
    mms2ut_half* cO = at<mms2ut_half>(A, off, MMS_SLOT_CO);
    mms2ut_half* xb = at<mms2ut_half>(A, off, MMS_SLOT_XB);
    if ((rc = mms2ut_layernorm_fwd(xa, L->ln2_g, L->ln2_b, h2, at<float>(A, off, MMS_SLOT_M2),
                                   at<float>(A, off, MMS_SLOT_R2), R, (int)d, L->eps, s))) return rc;
    if ((rc = linear(c, h2, L->w_cq, L->b_cq, q, R, d, d))) return rc;
    mms2ut_attn_args a = attn(q, d, L->kv, L->kv + d, L->ld_kv, cO, d, L->B, L->H, L->T, L->Tk, hd, L->cross_len, 0,
                              L->p_attn, L->seed, L->off_ca_attn, at<float>(A, off, MMS_SLOT_LSE_CA));
    if ((rc = mms2ut_mha_varlen_fwd(&a, s))) return rc;
    if ((rc = linear(c, cO, L->w_co, L->b_co, xb, R, d, d, MMS_EPI_DROP_RESID, xa, L->p_drop, L->seed,
                     L->off_ca_res))) return rc;
    xf = xb;
  }
  // FFN block: LN -> fc1 (+relu +dropout) -> fc2 (+dropout +residual)
  mms2ut_half* h3 = at<mms2ut_half>(A, off, MMS_SLOT_H3);
  mms2ut_half* f1 = at<mms2ut_half>(A, off, MMS_SLOT_F1);
  if ((rc = mms2ut_layernorm_fwd(xf, L->ln3_g, L->ln3_b, h3, at<float>(A, off, MMS_SLOT_M3),
                                 at<float>(A, off, MMS_SLOT_R3), R, (int)d, L->eps, s))) return rc;
  if ((rc = linear(c, h3, L->w_fc1, L->b_fc1, f1, R, F, d, MMS_EPI_RELU_DROP, nullptr, L->p_act, L->seed, L->off_act)))
    return rc;
  return linear(c, f1, L->w_fc2, L->b_fc2, at<mms2ut_half>(A, off, MMS_SLOT_OUT), R, d, F, MMS_EPI_DROP_RESID, xf,
                L->p_drop, L->seed, L->off_ffn_res);
}

extern "C" int mms2ut_layer_bwd(const mms2ut_layer* L, const mms2ut_layer_grad* G, hipStream_t main,
                                hipStream_t side) {
  MMS_REQUIRE(L && G && G->dy && G->scratch && L->saved, "layer_bwd: null layer / gradient / scratch / arena");
  MMS_REQUIRE(L->kind != MMS_LAYER_DEC || G->dkv, "layer_bwd: decoder needs dkv");
  if (!side) side = main;
  const Dims D = dims_of(L);
  int64_t sz[MMS_LAYER_NSLOT], off[MMS_LAYER_NSLOT], ssz[S_N], so[S_N];
  arena_sizes(D, sz);
  layout(sz, MMS_LAYER_NSLOT, off);
  scratch_sizes(D, G->emit_p, ssz);
  layout(ssz, S_N, so);
  void* A = L->saved;
  void* S = G->scratch;
  const int64_t R = D.R, d = D.d, F = D.F;
  mms2ut_wgrad group[8];
  int ngroup = 0;
  const Ctx c{main, side, G->main_ws, G->main_ws_floats, G->side_ws, G->side_ws_floats, at<float>(S, so, S_BPART),
              group, &ngroup, group_ok(D)};
  const int hd = L->d / L->H, Dm = (int)d;
  const float pd = L->p_drop;
  int rc;
  auto H_ = [&](int slot) { return at<mms2ut_half>(A, off, slot); };
  auto F_ = [&](int slot) { return at<float>(A, off, slot); };
  auto SH = [&](int slot) { return at<mms2ut_half>(S, so, slot); };
  auto SF = [&](int slot) { return at<float>(S, so, slot); };
  const mms2ut_half* xf = D.dec ? H_(MMS_SLOT_XB) : H_(MMS_SLOT_XA);
  // ---- FFN block.  dyd = dropout(dy) with the fc2 residual mask (from the layer above, or here)
  const mms2ut_half* dyd = G->dy_drop;
  if (!dyd) {
    if (pd > 0.f) {
      if ((rc = mms2ut_dropout_fwd(G->dy, SH(S_DYD), R * d, pd, L->seed, L->off_ffn_res, main))) return rc;
      dyd = SH(S_DYD);
    } else {
      dyd = G->dy;
    }
  }
  if ((rc = dgrad(c, dyd, d, L->w_fc2, L->wt_fc2, SH(S_DF1), R, d, F, MMS_EPI_RELU_DROP_BWD, H_(MMS_SLOT_F1),
                  L->p_act))) return rc;
  // the layer above's deferred weight gradients, launched at flush point MMS2UT_WGRAD_DEFER of this
  // layer (1: after this first dgrad, 2: after fc1's dgrad, 3: after LN3, 4: after the next
  // out-projection dgrad, 5: after the self-attention backward, 6: after the QKV dgrad)
  const int fp = wgrad_defer_mode();
  auto flush_at = [&](int point) { return point == fp ? flush_pending(main) : 0; };
  if ((rc = flush_at(1))) return rc;
  if ((rc = wgrad(c, dyd, d, H_(MMS_SLOT_F1), F, L->g_w_fc2, L->g_b_fc2, R, d, F))) return rc;
  if ((rc = dgrad(c, SH(S_DF1), F, L->w_fc1, L->wt_fc1, SH(S_DH3), R, F, d)) || (rc = flush_at(2))) return rc;
  if ((rc = wgrad(c, SH(S_DF1), F, H_(MMS_SLOT_H3), d, L->g_w_fc1, L->g_b_fc1, R, F, d))) return rc;
  if (c.grouped && wgrad_split_mode()) {
    // A/B (MMS2UT_WGRAD_SPLIT=1): the FFN weight gradients as their own grouped launch right here,
    // beside the rest of this layer's (attention / LayerNorm) backward instead of the next layer's
    // FFN dgrads; the attention projections' group follows at the end as usual
    if ((rc = fork(c)) || (rc = mms2ut_wgrad_group(group, ngroup, R, side == main ? 0 : G->side_blocks, side))) return rc;
    ngroup = 0;
  }
  // LN3 backward: dx of the FFN input (+ the residual dy) and its dropout with the mask of the
  // block below's residual branch (cross-attention for the decoder, self-attention for the encoder)
  mms2ut_half* dxf = D.dec ? SH(S_DX3) : SH(S_DX2);
  const uint64_t below_off = D.dec ? L->off_ca_res : L->off_sa_res;
  if ((rc = ln_bwd(c, SH(S_DH3), xf, L->ln3_g, F_(MMS_SLOT_M3), F_(MMS_SLOT_R3), G->dy, dxf, SH(S_DY3B), pd, L->seed,
                   below_off, SF(S_P3), L->g_ln3, R, Dm)) || (rc = flush_at(3))) return rc;
  const mms2ut_half* dbr = pd > 0.f ? SH(S_DY3B) : dxf;   // the block below's residual-branch gradient
  mms2ut_half* dxa = SH(S_DX2);                            // gradient of the self-attention block output
  if (D.dec) {
    // ---- cross-attention block
    if ((rc = dgrad(c, dbr, d, L->w_co, L->wt_co, SH(S_DO2), R, d, d))) return rc;
    if ((rc = wgrad(c, dbr, d, H_(MMS_SLOT_CO), d, L->g_w_co, L->g_b_co, R, d, d))) return rc;
    mms2ut_attn_args a = attn(H_(MMS_SLOT_Q), d, L->kv, L->kv + d, L->ld_kv, H_(MMS_SLOT_CO), d, L->B, L->H, L->T, L->Tk,
                              hd, L->cross_len, 0, L->p_attn, L->seed, L->off_ca_attn, F_(MMS_SLOT_LSE_CA));
    if ((rc = mms2ut_mha_varlen_bwd(&a, SH(S_DO2), d, 0, SF(S_DD_CA), SH(S_DQ), d, 0, G->dkv, G->ld_dkv, 0,
                                    G->dkv + d, G->ld_dkv, 0, main))) return rc;
    if ((rc = dgrad(c, SH(S_DQ), d, L->w_cq, L->wt_cq, SH(S_DH2), R, d, d))) return rc;
    if ((rc = wgrad(c, SH(S_DQ), d, H_(MMS_SLOT_H2), d, L->g_w_cq, L->g_b_cq, R, d, d))) return rc;
    if ((rc = ln_bwd(c, SH(S_DH2), H_(MMS_SLOT_XA), L->ln2_g, F_(MMS_SLOT_M2), F_(MMS_SLOT_R2), dxf, dxa, SH(S_DY2B),
                     pd, L->seed, L->off_sa_res, SF(S_P2), L->g_ln2, R, Dm))) return rc;
    dbr = pd > 0.f ? SH(S_DY2B) : dxa;
  }
  // ---- self-attention block
  if ((rc = dgrad(c, dbr, d, L->w_o, L->wt_o, SH(S_DO), R, d, d)) || (rc = flush_at(4))) return rc;
  if ((rc = wgrad(c, dbr, d, H_(MMS_SLOT_O), d, L->g_w_o, L->g_b_o, R, d, d))) return rc;
  {
    mms2ut_half* qkv = H_(MMS_SLOT_QKV);
    mms2ut_half* dqkv = SH(S_DQKV);
    mms2ut_attn_args a = attn(qkv, 3 * d, qkv + d, qkv + 2 * d, 3 * d, H_(MMS_SLOT_O), d, L->B, L->H, L->T, L->T, hd,
                              L->self_len, D.dec ? 1 : 0, L->p_attn, L->seed, L->off_sa_attn, F_(MMS_SLOT_LSE_SA));
    if ((rc = mms2ut_mha_varlen_bwd(&a, SH(S_DO), d, 0, SF(S_DD_SA), dqkv, 3 * d, 0, dqkv + d, 3 * d, 0, dqkv + 2 * d,
                                    3 * d, 0, main)) || (rc = flush_at(5))) return rc;
    if ((rc = dgrad(c, dqkv, 3 * d, L->w_qkv, L->wt_qkv, SH(S_DH1), R, 3 * d, d)) || (rc = flush_at(6))) return rc;
    if ((rc = wgrad(c, dqkv, 3 * d, H_(MMS_SLOT_H1), d, L->g_w_qkv, L->g_b_qkv, R, 3 * d, d))) return rc;
  }
  // LN1 backward: the layer input's gradient (+ dropout for the layer below when asked)
  if ((rc = ln_bwd(c, SH(S_DH1), L->x, L->ln1_g, F_(MMS_SLOT_M1), F_(MMS_SLOT_R1), dxa, SH(S_DX), SH(S_DXD), G->emit_p,
                   G->emit_seed, G->emit_offset, SF(S_P1), L->g_ln1, R, Dm))) return rc;
  if ((rc = flush_pending(main))) return rc;   // a flush point past this layer's last one
  if (!c.grouped || ngroup == 0) return 0;
  if (wgrad_defer_mode() && side != main) {
    g_pend.on = true;
    std::copy(group, group + ngroup, g_pend.w);
    g_pend.n = ngroup;
    g_pend.rows = R;
    g_pend.blocks = G->side_blocks;
    g_pend.side = side;
    return 0;
  }
  // the layer's weight gradients: one grouped launch on the side stream, behind everything the
  // main stream enqueued for this layer (it overlaps the next layer's dgrad chain)
  if ((rc = fork(c))) return rc;
  return mms2ut_wgrad_group(group, ngroup, R, side == main ? 0 : G->side_blocks, side);
}

extern "C" int mms2ut_wgrad_flush(hipStream_t main) { return flush_pending(main); }

// ---------------------------------------------------------------- Conv1d subsampler (one call)
// fairseq Conv1dSubsampler (S2TTransformerEncoder's front, reached at mm_s2s_transformer.py:464):
// nlayers x [Conv1d(C_l -> cout_l, k_l, stride 2, padding k_l / 2) -> GLU(dim = channels)], as
// implicit GEMMs: im2col (K = C_l k_l, padded to whole 64-wide k-tiles with zero columns and a
// zero-padded copy of the weight when C_l k_l % 64 != 0), the projection GEMM with its bias, the
// GLU.  The same kernels / arguments / stream order as the per-launch path (model.subsample_*_ref),
// so results are bit-identical to it (tests/test_gpu_layers.py).
namespace {

struct ConvDims {
  int n;
  int64_t Tin[MMS_CONV_MAX], Tout[MMS_CONV_MAX], C[MMS_CONV_MAX], ck[MMS_CONV_MAX], kp[MMS_CONV_MAX];
  int64_t rows[MMS_CONV_MAX];
};

ConvDims conv_dims(const mms2ut_conv1d_glu* c) {
  ConvDims D{};
  D.n = c->nlayers;
  int64_t T = c->T, C = c->C;
  for (int i = 0; i < D.n; ++i) {
    D.Tin[i] = T;
    D.Tout[i] = (T - 1) / 2 + 1;
    D.C[i] = C;
    D.ck[i] = C * c->k[i];
    D.kp[i] = D.ck[i] % 64 ? (D.ck[i] + 63) / 64 * 64 : D.ck[i];
    D.rows[i] = (int64_t)c->B * D.Tout[i];
    T = D.Tout[i];
    C = c->cout[i] / 2;
  }
  return D;
}

// arena: per layer col, y (pre-GLU), g (GLU output = the next layer's input / the result), Wp
enum { CA_COL = 0, CA_Y, CA_G, CA_WP, CA_N };
void conv_arena_sizes(const mms2ut_conv1d_glu* c, const ConvDims& D, int64_t* sz) {
  for (int i = 0; i < MMS_CONV_MAX * CA_N; ++i) sz[i] = 0;
  for (int i = 0; i < D.n; ++i) {
    sz[i * CA_N + CA_COL] = D.rows[i] * D.kp[i] * 2;
    sz[i * CA_N + CA_Y] = D.rows[i] * c->cout[i] * 2;
    sz[i * CA_N + CA_G] = D.rows[i] * (c->cout[i] / 2) * 2;
    sz[i * CA_N + CA_WP] = D.kp[i] != D.ck[i] ? (int64_t)c->cout[i] * D.kp[i] * 2 : 0;
  }
}
// scratch: per layer dy (pre-GLU gradient), dcol, dx (the layer input's gradient; layers > 0), and
// the colsum partials of the bias-gradient fallback
enum { CS_DY = 0, CS_DCOL, CS_DX, CS_N };
void conv_scratch_sizes(const mms2ut_conv1d_glu* c, const ConvDims& D, int64_t* sz) {
  for (int i = 0; i < MMS_CONV_MAX * CS_N + 1; ++i) sz[i] = 0;
  int64_t maxc = 0;
  for (int i = 0; i < D.n; ++i) {
    sz[i * CS_N + CS_DY] = D.rows[i] * c->cout[i] * 2;
    if (i > 0) {
      sz[i * CS_N + CS_DCOL] = D.rows[i] * D.ck[i] * 2;
      sz[i * CS_N + CS_DX] = (int64_t)c->B * D.Tin[i] * D.C[i] * 2;
    }
    maxc = std::max<int64_t>(maxc, c->cout[i]);
  }
  sz[MMS_CONV_MAX * CS_N] = (int64_t)mms2ut_colsum_nparts(D.rows[0]) * maxc * 4;
}

bool conv_group_ok(const mms2ut_conv1d_glu* c, const ConvDims& D, int i) {
  // kernels.linear_wgrad: >= 256 output tiles and the grouped kernel's shape rules -> unsplit grouped
  const int64_t N = c->cout[i], Kk = D.ck[i];
  return ((N + 127) / 128) * ((Kk + 127) / 128) >= 256 && N % 8 == 0 && Kk % 8 == 0 && D.kp[i] % 8 == 0 &&
         D.rows[i] * std::max<int64_t>(N, D.kp[i]) * 2 < (1LL << 31);
}

int conv_check(const mms2ut_conv1d_glu* c) {
  MMS_REQUIRE(c && c->nlayers >= 1 && c->nlayers <= MMS_CONV_MAX, "conv1d_glu: 1..%d layers", MMS_CONV_MAX);
  MMS_REQUIRE(c->B >= 0 && c->T >= 1 && c->C >= 1, "conv1d_glu: B=%d T=%d C=%d", c->B, c->T, c->C);
  for (int i = 0; i < c->nlayers; ++i)
    MMS_REQUIRE(c->k[i] >= 1 && c->cout[i] > 0 && c->cout[i] % 16 == 0 && c->w[i] && c->b[i],
                "conv1d_glu: layer %d: k=%d cout=%d (multiple of 16), weight and bias required", i, c->k[i], c->cout[i]);
  return 0;
}

}  // namespace

extern "C" int mms2ut_conv1d_glu_arena(const mms2ut_conv1d_glu* c, int64_t* out_offset, int64_t* bytes) {
  if (int rc = conv_check(c)) return rc;
  MMS_REQUIRE(bytes, "conv1d_glu_arena: null");
  const ConvDims D = conv_dims(c);
  int64_t sz[MMS_CONV_MAX * CA_N], off[MMS_CONV_MAX * CA_N];
  conv_arena_sizes(c, D, sz);
  *bytes = layout(sz, MMS_CONV_MAX * CA_N, off);
  if (out_offset) *out_offset = off[(D.n - 1) * CA_N + CA_G];
  return 0;
}

extern "C" int mms2ut_conv1d_glu_scratch(const mms2ut_conv1d_glu* c, int64_t* dx_offset, int64_t* bytes) {
  if (int rc = conv_check(c)) return rc;
  MMS_REQUIRE(bytes, "conv1d_glu_scratch: null");
  const ConvDims D = conv_dims(c);
  int64_t sz[MMS_CONV_MAX * CS_N + 1], off[MMS_CONV_MAX * CS_N + 1];
  conv_scratch_sizes(c, D, sz);
  *bytes = layout(sz, MMS_CONV_MAX * CS_N + 1, off);
  if (dx_offset) *dx_offset = D.n > 1 ? off[1 * CS_N + CS_DX] : -1;   // gradient of layer 1's input
  return 0;
}

extern "C" int mms2ut_conv1d_glu_ws(const mms2ut_conv1d_glu* c, int64_t* main_floats, int64_t* side_floats) {
  if (int rc = conv_check(c)) return rc;
  MMS_REQUIRE(main_floats && side_floats, "conv1d_glu_ws: null");
  const ConvDims D = conv_dims(c);
  int64_t mw = 0, sw = 0;
  for (int i = 0; i < D.n; ++i) {
    const int64_t N = c->cout[i];
    int s = fixup_splits(D.rows[i], N, D.kp[i]);
    if (s > 1) mw = std::max(mw, (int64_t)s * D.rows[i] * N);
    if (i > 0 && (s = fixup_splits(D.rows[i], D.ck[i], N)) > 1) mw = std::max(mw, (int64_t)s * D.rows[i] * D.ck[i]);
    if (!conv_group_ok(c, D, i)) {
      s = wgrad_splits(((N + 127) / 128) * ((D.ck[i] + 127) / 128), D.rows[i]);
      sw = std::max(sw, (int64_t)s * N * D.ck[i] + (int64_t)s * N);
    }
  }
  *main_floats = mw;
  *side_floats = sw;
  return 0;
}

extern "C" int mms2ut_conv1d_glu_fwd(const mms2ut_conv1d_glu* c, float* main_ws, int64_t main_ws_floats,
                                     hipStream_t s) {
  if (int rc = conv_check(c)) return rc;
  MMS_REQUIRE(c->x && c->saved, "conv1d_glu_fwd: null input / arena");
  const ConvDims D = conv_dims(c);
  int64_t sz[MMS_CONV_MAX * CA_N], off[MMS_CONV_MAX * CA_N];
  conv_arena_sizes(c, D, sz);
  layout(sz, MMS_CONV_MAX * CA_N, off);
  void* A = c->saved;
  const Ctx cx{s, s, main_ws, main_ws_floats, nullptr, 0, nullptr};
  const mms2ut_half* x = c->x;
  int rc;
  for (int i = 0; i < D.n; ++i) {
    const int k = c->k[i], N = c->cout[i];
    mms2ut_half* col = at<mms2ut_half>(A, off, i * CA_N + CA_COL);
    mms2ut_half* y = at<mms2ut_half>(A, off, i * CA_N + CA_Y);
    mms2ut_half* g = at<mms2ut_half>(A, off, i * CA_N + CA_G);
    if ((rc = mms2ut_im2col_ld(x, col, c->B, (int)D.Tin[i], (int)D.Tout[i], (int)D.C[i], k, 2, k / 2, (int)D.kp[i], s)))
      return rc;
    const mms2ut_half* W = c->w[i];
    if (D.kp[i] != D.ck[i]) {   // the weight, zero-padded to the padded K
      mms2ut_half* Wp = at<mms2ut_half>(A, off, i * CA_N + CA_WP);
      if ((rc = mms2ut_copy2d_pad(W, D.ck[i], Wp, D.kp[i], N, (int)D.ck[i], (int)(D.kp[i] - D.ck[i]), s))) return rc;
      W = Wp;
    }
    if ((rc = linear(cx, col, W, c->b[i], y, D.rows[i], N, D.kp[i]))) return rc;
    if ((rc = mms2ut_glu_fwd(y, g, D.rows[i], N / 2, s))) return rc;
    x = g;
  }
  return 0;
}

extern "C" int mms2ut_conv1d_glu_bwd(const mms2ut_conv1d_glu* c, const mms2ut_half* dy, void* scratch,
                                     float* main_ws, int64_t main_ws_floats, float* side_ws,
                                     int64_t side_ws_floats, int side_blocks, hipStream_t main, hipStream_t side) {
  if (int rc = conv_check(c)) return rc;
  MMS_REQUIRE(dy && scratch && c->saved, "conv1d_glu_bwd: null gradient / scratch / arena");
  if (!side) side = main;
  const ConvDims D = conv_dims(c);
  int64_t sz[MMS_CONV_MAX * CA_N], off[MMS_CONV_MAX * CA_N];
  conv_arena_sizes(c, D, sz);
  layout(sz, MMS_CONV_MAX * CA_N, off);
  int64_t ssz[MMS_CONV_MAX * CS_N + 1], so[MMS_CONV_MAX * CS_N + 1];
  conv_scratch_sizes(c, D, ssz);
  layout(ssz, MMS_CONV_MAX * CS_N + 1, so);
  void* A = c->saved;
  void* S = scratch;
  const Ctx cx{main, side, main_ws, main_ws_floats, side_ws, side_ws_floats, at<float>(S, so, MMS_CONV_MAX * CS_N),
               nullptr, nullptr, false};
  const mms2ut_half* dg = dy;   // gradient of layer i's GLU output
  int rc;
  for (int i = D.n - 1; i >= 0; --i) {
    const int k = c->k[i], N = c->cout[i];
    const mms2ut_half* col = at<mms2ut_half>(A, off, i * CA_N + CA_COL);
    mms2ut_half* dyi = at<mms2ut_half>(S, so, i * CS_N + CS_DY);
    if ((rc = mms2ut_glu_bwd(at<mms2ut_half>(A, off, i * CA_N + CA_Y), dg, dyi, D.rows[i], N / 2, main))) return rc;
    // dW [N, C k] (the weight's [out][C][k] layout) and db: on the side stream
    if (c->g_w[i]) {
      if (conv_group_ok(c, D, i)) {
        if ((rc = fork(cx))) return rc;
        mms2ut_wgrad w{dyi, N, col, D.kp[i], c->g_w[i], c->g_b[i], N, (int)D.ck[i]};
        if ((rc = mms2ut_wgrad_group(&w, 1, D.rows[i], side == main ? 0 : side_blocks, side))) return rc;
      } else if ((rc = wgrad(cx, dyi, N, col, D.kp[i], c->g_w[i], c->g_b[i], D.rows[i], N, D.ck[i]))) {
        return rc;
      }
    }
    if (i == 0) break;
    mms2ut_half* dcol = at<mms2ut_half>(S, so, i * CS_N + CS_DCOL);
    mms2ut_half* dx = at<mms2ut_half>(S, so, i * CS_N + CS_DX);
    if ((rc = dgrad(cx, dyi, N, c->w[i], c->wt[i], dcol, D.rows[i], N, D.ck[i]))) return rc;
    if ((rc = mms2ut_col2im(dcol, dx, c->B, (int)D.Tin[i], (int)D.Tout[i], (int)D.C[i], k, 2, k / 2, main))) return rc;
    dg = dx;
  }
  return 0;
}

// ---------------------------------------------------------------- gated fusion (one call)
// The reference fusion tail (fuse_img_feat, mm_s2s_transformer.py:594-622; fuse.py:65-117
// SelectiveAttention / fuse.py:145-167 MultimodalAttention = nn.MultiheadAttention with
// add_bias_kv) behind SURVEY §8b mms2ut_gated_fusion_{fwd,bwd}: image LayerNorm (+ SA_image
// dropout, laid out as [B][Ti (+1 bias_kv row)][Di] keys), text dropout, q / k|v projections, one-head
// attention over the image keys (scores materialised: hd = d is past the flash kernel's head
// sizes), out-projection, and the sigmoid gate merge (or the plain residual without the gate).
// The launch sequence, arguments and stream order are model.fusion_fwd_ref / fusion_bwd_ref's, so
// results are bit-identical to that per-launch path (tests/test_gpu_layers.py).
namespace {

// kernels.linear_wgrad's choice: the grouped unsplit kernel for >= 256 output tiles whose shapes
// it takes, else fp32 split-K slabs (wgrad above); both on the side stream
bool wgrad_group_ok(const mms2ut_half* dy, int64_t lddy, const mms2ut_half* x, int64_t ldx, const mms2ut_half* dW,
                    int64_t M, int64_t N, int64_t K) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return ((N + 127) / 128) * ((K + 127) / 128) >= 256 && N % 8 == 0 && K % 8 == 0 && lddy % 8 == 0 && ldx % 8 == 0 &&
         al16(dy) && al16(x) && al16(dW) && M * std::max(lddy, ldx) * 2 < (1LL << 31);
}

int wgrad_auto(const Ctx& c, const mms2ut_half* dy, int64_t lddy, const mms2ut_half* x, int64_t ldx, mms2ut_half* dW,
               mms2ut_half* db, int64_t M, int64_t N, int64_t K, int side_blocks) {
  if (wgrad_group_ok(dy, lddy, x, ldx, dW, M, N, K)) {
    int rc = fork(c);
    if (rc) return rc;
    mms2ut_wgrad w{dy, lddy, x, ldx, dW, db, (int)N, (int)K};
    return mms2ut_wgrad_group(&w, 1, M, c.side == c.main ? 0 : side_blocks, c.side);
  }
  return wgrad(c, dy, lddy, x, ldx, dW, db, M, N, K);
}

struct FusDims {
  int64_t B, Te, Ti, Tk, Di, d, Rt, Ri, Rk, ldS;
  bool extra, gate, pre, ln_fused;
};

FusDims fus_dims(const mms2ut_gated_fusion* f) {
  FusDims D;
  D.B = f->B; D.Te = f->Te; D.Ti = f->Ti; D.Di = f->Di; D.d = f->d;
  D.extra = f->extra != 0; D.gate = f->gate != 0; D.pre = f->image_pre_norm != 0;
  D.Tk = D.Ti + (D.extra ? 1 : 0);
  D.Rt = D.B * D.Te; D.Ri = D.B * D.Ti; D.Rk = D.B * D.Tk;
  D.ldS = (D.Tk + 7) / 8 * 8;
  D.ln_fused = D.pre && D.Di % 256 == 0 && D.Di <= 1024;
  return D;
}

enum { FA_IM = 0, FA_IR, FA_IMGN, FA_IMGD, FA_TEXTD, FA_Q, FA_KV, FA_S, FA_P, FA_PD, FA_O, FA_MERGE, FA_G, FA_OUT, FA_N };
void fus_arena_sizes(const mms2ut_gated_fusion* f, const FusDims& D, int64_t* sz) {
  for (int i = 0; i < FA_N; ++i) sz[i] = 0;
  const int64_t h = 2;
  if (D.pre) sz[FA_IM] = sz[FA_IR] = D.Ri * 4;
  if (!D.ln_fused && (D.pre || f->p_img > 0.f)) sz[FA_IMGN] = D.Ri * D.Di * h;
  if (D.ln_fused || D.extra) sz[FA_IMGD] = D.Rk * D.Di * h;
  if (f->p_txt > 0.f) sz[FA_TEXTD] = D.Rt * D.d * h;
  sz[FA_Q] = D.Rt * D.d * h;
  sz[FA_KV] = D.Rk * 2 * D.d * h;
  sz[FA_S] = sz[FA_P] = D.Rt * D.ldS * h;
  if (f->p_attn > 0.f) sz[FA_PD] = sz[FA_P];
  sz[FA_O] = D.Rt * D.d * h;
  if (D.gate) { sz[FA_MERGE] = D.Rt * 2 * D.d * h; sz[FA_G] = D.Rt * D.d * h; }
  sz[FA_OUT] = D.Rt * D.d * h;
}

enum { FS_DPRE = 0, FS_DMERGE, FS_DO, FS_DQ, FS_DKV, FS_DPD, FS_DIMGD, FS_DIMG, FS_DIMGIN, FS_DTEXT, FS_LNP, FS_KVP,
       FS_BPART, FS_N };
void fus_scratch_sizes(const mms2ut_gated_fusion* f, const FusDims& D, int want_dimg, int64_t* sz) {
  for (int i = 0; i < FS_N; ++i) sz[i] = 0;
  const int64_t h = 2;
  if (D.gate) { sz[FS_DPRE] = D.Rt * D.d * h; sz[FS_DMERGE] = D.Rt * 2 * D.d * h; }
  sz[FS_DO] = sz[FS_DQ] = D.Rt * D.d * h;
  sz[FS_DKV] = D.Rk * 2 * D.d * h;
  sz[FS_DPD] = D.Rt * D.ldS * h;
  if (D.pre || want_dimg) {
    sz[FS_DIMGD] = D.Rk * D.Di * h;
    sz[FS_DIMG] = D.Ri * D.Di * h;
    sz[FS_DIMGIN] = D.Ri * D.Di * h;
    if (D.pre) sz[FS_LNP] = (int64_t)mms2ut_layernorm_bwd_nparts(D.Ri, (int)D.Di) * 2 * D.Di * 4;
  }
  sz[FS_DTEXT] = D.Rt * D.d * h;
  if (D.extra) sz[FS_KVP] = (int64_t)mms2ut_colsum_nparts(D.B) * 2 * D.d * 4;
  sz[FS_BPART] = (int64_t)mms2ut_colsum_nparts(std::max(D.Rt, D.Rk)) * 2 * D.d * 4;
}

int fus_check(const mms2ut_gated_fusion* f) {
  MMS_REQUIRE(f && f->B >= 1 && f->Te >= 1 && f->Ti >= 1, "gated_fusion: B, Te, Ti must be >= 1");
  MMS_REQUIRE(f->d % 8 == 0 && f->Di % 8 == 0 && f->d > 0 && f->Di > 0, "gated_fusion: d=%d Di=%d (multiples of 8)", f->d, f->Di);
  MMS_REQUIRE(f->wq && f->bq && f->wkv && f->bkv && f->wo && f->bo, "gated_fusion: projection weights / biases required");
  MMS_REQUIRE(!f->extra || f->bias_kv, "gated_fusion: multimodal attention needs bias_kv");
  MMS_REQUIRE(!f->gate || (f->wg && f->bg), "gated_fusion: the gate needs its weight and bias");
  MMS_REQUIRE(!f->image_pre_norm || (f->ln_g && f->ln_b), "gated_fusion: image_pre_norm needs the LayerNorm");
  return 0;
}

mms2ut_gemm_args batched(const mms2ut_half* A, const mms2ut_half* B_, void* C, int M, int N, int K, int a_kc, int b_kc,
                         int64_t lda, int64_t ldb, int64_t ldc, int batch, int64_t sA, int64_t sB, int64_t sC,
                         float alpha) {
  // model.attn_fwd / attn_bwd's batched products (H = 1: bdiv 1, the head strides unused)
  mms2ut_gemm_args a = gemm_args();
  a.A = A; a.B = B_; a.C = C;
  a.M = M; a.N = N; a.K = K;
  a.a_kcontig = a_kc; a.b_kcontig = b_kc;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.batch = batch; a.bdiv = 1;
  a.sA1 = sA; a.sB1 = sB; a.sC1 = sC;
  a.sA2 = a.sB2 = a.sC2 = 0;
  a.alpha = alpha;
  return a;
}

int zero_rows(mms2ut_half* p, int64_t pitch_elems, int64_t width_elems, int64_t rows, hipStream_t s) {
  return mms2ut_copy2d_pad(nullptr, 0, p, pitch_elems, rows, 0, (int)width_elems, s);
}

}  // namespace

extern "C" int mms2ut_gated_fusion_arena(const mms2ut_gated_fusion* f, int64_t* out_offset, int64_t* bytes) {
  if (int rc = fus_check(f)) return rc;
  MMS_REQUIRE(bytes, "gated_fusion_arena: null");
  const FusDims D = fus_dims(f);
  int64_t sz[FA_N], off[FA_N];
  fus_arena_sizes(f, D, sz);
  *bytes = layout(sz, FA_N, off);
  if (out_offset) *out_offset = off[FA_OUT];
  return 0;
}

extern "C" int mms2ut_gated_fusion_scratch(const mms2ut_gated_fusion* f, int want_dimg, int64_t* offsets, int64_t* bytes) {
  if (int rc = fus_check(f)) return rc;
  MMS_REQUIRE(bytes, "gated_fusion_scratch: null");
  const FusDims D = fus_dims(f);
  int64_t sz[FS_N], off[FS_N];
  fus_scratch_sizes(f, D, want_dimg, sz);
  *bytes = layout(sz, FS_N, off);
  if (offsets) {
    offsets[0] = off[FS_DTEXT];
    // the image gradient: LN backward's dx, or the (un-padded, dropout-applied) key gradient
    offsets[1] = want_dimg ? (D.pre ? off[FS_DIMGIN] : (D.extra ? off[FS_DIMG] : off[FS_DIMGD])) : -1;
  }
  return 0;
}

extern "C" int mms2ut_gated_fusion_ws(const mms2ut_gated_fusion* f, int64_t* main_floats, int64_t* side_floats) {
  if (int rc = fus_check(f)) return rc;
  MMS_REQUIRE(main_floats && side_floats, "gated_fusion_ws: null");
  const FusDims D = fus_dims(f);
  int64_t mw = 0, sw = 0;
  auto fw = [&](int64_t M, int64_t N, int64_t K) {
    const int s = fixup_splits(M, N, K);
    if (s > 1) mw = std::max(mw, (int64_t)s * M * N);
  };
  auto ww = [&](int64_t M, int64_t N, int64_t K) {
    const int s = wgrad_splits(((N + 127) / 128) * ((K + 127) / 128), M);
    sw = std::max(sw, (int64_t)s * N * K + (int64_t)s * N);
  };
  const int64_t d = D.d;
  fw(D.Rt, d, d); fw(D.Rk, 2 * d, D.Di); fw(D.Rt, d, d); fw(D.Rt, d, 2 * d);      // forward
  fw(D.Rt, 2 * d, d); fw(D.Rt, d, d); fw(D.Rk, D.Di, 2 * d); fw(D.Rt, d, d);      // dgrads
  ww(D.Rt, d, 2 * d); ww(D.Rt, d, d); ww(D.Rk, 2 * d, D.Di); ww(D.Rt, d, d);      // weight gradients
  *main_floats = mw;
  *side_floats = sw;
  return 0;
}

extern "C" int mms2ut_gated_fusion_fwd(const mms2ut_gated_fusion* f, float* main_ws, int64_t main_ws_floats,
                                       hipStream_t s) {
  if (int rc = fus_check(f)) return rc;
  MMS_REQUIRE(f->text && f->img && f->saved, "gated_fusion_fwd: null text / image / arena");
  const FusDims D = fus_dims(f);
  int64_t sz[FA_N], off[FA_N];
  fus_arena_sizes(f, D, sz);
  layout(sz, FA_N, off);
  void* A = f->saved;
  auto H_ = [&](int slot) { return at<mms2ut_half>(A, off, slot); };
  const Ctx c{s, s, main_ws, main_ws_floats, nullptr, 0, nullptr};
  const int64_t d = D.d, Di = D.Di;
  int rc;
  // image: LayerNorm (+ dropout) into the [B][Tk][Di] key layout (bias_kv row zero)
  const mms2ut_half* imgd;
  if (D.ln_fused) {
    if (D.extra && (rc = zero_rows(H_(FA_IMGD) + D.Ti * Di, D.Tk * Di, Di, D.B, s))) return rc;
    if ((rc = mms2ut_layernorm_fwd_ex(f->img, f->ln_g, f->ln_b, H_(FA_IMGD), at<float>(A, off, FA_IM),
                                      at<float>(A, off, FA_IR), D.Ri, (int)Di, f->eps, D.extra ? D.Ti : 0,
                                      D.extra ? D.Tk : 0, f->p_img, f->seed, f->off_img, s))) return rc;
    imgd = H_(FA_IMGD);
  } else {
    const mms2ut_half* imgn = f->img;
    if (D.pre) {
      if ((rc = mms2ut_layernorm_fwd(f->img, f->ln_g, f->ln_b, H_(FA_IMGN), at<float>(A, off, FA_IM),
                                     at<float>(A, off, FA_IR), D.Ri, (int)Di, f->eps, s))) return rc;
      imgn = H_(FA_IMGN);
    }
    if (f->p_img > 0.f) {
      if ((rc = mms2ut_dropout_fwd(imgn, H_(FA_IMGN), D.Ri * Di, f->p_img, f->seed, f->off_img, s))) return rc;
      imgn = H_(FA_IMGN);
    }
    if (D.extra) {
      // the image rows and the zero bias_kv row of every batch entry in one pass
      if ((rc = mms2ut_copy2d_pad(imgn, D.Ti * Di, H_(FA_IMGD), D.Tk * Di, D.B, (int)(D.Ti * Di),
                                  (int)((D.Tk - D.Ti) * Di), s)))
        return rc;
      imgd = H_(FA_IMGD);
    } else {
      imgd = imgn;
    }
  }
  const mms2ut_half* textd = f->text;
  if (f->p_txt > 0.f) {
    if ((rc = mms2ut_dropout_fwd(f->text, H_(FA_TEXTD), D.Rt * d, f->p_txt, f->seed, f->off_txt, s))) return rc;
    textd = H_(FA_TEXTD);
  }
  mms2ut_half *q = H_(FA_Q), *kv = H_(FA_KV), *O = H_(FA_O);
  if ((rc = linear(c, textd, f->wq, f->bq, q, D.Rt, d, d))) return rc;
  if ((rc = linear(c, imgd, f->wkv, f->bkv, kv, D.Rk, 2 * d, Di))) return rc;
  if (D.extra && (rc = mms2ut_copy2d(f->bias_kv, 0, kv + D.Ti * 2 * d, D.Tk * 2 * d, D.B, (int)(2 * d), s))) return rc;
  // one-head attention, scores materialised (model.attn_fwd)
  const float scale = (float)pow((double)d, -0.5);
  mms2ut_half *S = H_(FA_S), *P = H_(FA_P), *Pd = f->p_attn > 0.f ? H_(FA_PD) : P;
  {
    mms2ut_gemm_args a = batched(q, kv, S, (int)D.Te, (int)D.Tk, (int)d, 1, 1, d, 2 * d, D.ldS, (int)D.B, D.Te * d,
                                 D.Tk * 2 * d, D.Te * D.ldS, scale);
    if ((rc = mms2ut_gemm_f16(&a, s))) return rc;
  }
  if ((rc = mms2ut_attn_softmax_fwd(S, P, Pd, (int)D.B, 1, (int)D.Te, (int)D.Tk, D.ldS, nullptr, f->key_mask,
                                    f->key_mask ? f->ld_mask : 0, 0, D.extra ? 1 : 0, f->p_attn,
                                    f->p_attn > 0.f ? f->seed : 0, f->p_attn > 0.f ? f->off_attn : 0, s))) return rc;
  {
    mms2ut_gemm_args a = batched(Pd, kv + d, O, (int)D.Te, (int)d, (int)D.Tk, 1, 0, D.ldS, 2 * d, d, (int)D.B,
                                 D.Te * D.ldS, D.Tk * 2 * d, D.Te * d, 1.f);
    if ((rc = mms2ut_gemm_f16(&a, s))) return rc;
  }
  mms2ut_half* out = H_(FA_OUT);
  if (D.gate) {
    mms2ut_half* merge = H_(FA_MERGE);
    if ((rc = gemm_nt(c, O, d, f->wo, d, 1, merge, 2 * d, D.Rt, d, d, MMS_EPI_F16, f->bo, nullptr, 0, 0.f, 0, 0, d)))
      return rc;
    if ((rc = mms2ut_copy2d(textd, d, merge + d, 2 * d, D.Rt, (int)d, s))) return rc;
    mms2ut_gemm_args a = gemm_args();
    a.A = merge; a.B = f->wg; a.C = out;
    a.M = (int)D.Rt; a.N = (int)d; a.K = (int)(2 * d);
    a.a_kcontig = 1; a.b_kcontig = 1;
    a.lda = 2 * d; a.ldb = 2 * d; a.ldc = d;
    a.epi = MMS_EPI_GATE; a.bias = f->bg; a.aux = merge; a.ldaux = 2 * d; a.out2 = H_(FA_G); a.ldo2 = d;
    a.ld_rng = d;
    const int sp = fixup_splits(D.Rt, d, 2 * d);
    if (sp > 1) {
      MMS_REQUIRE(main_ws && main_ws_floats >= (int64_t)sp * D.Rt * d, "gated_fusion_fwd: main workspace too small");
      a.splitk = sp; a.splitk_ws = main_ws; a.splitk_ws_floats = main_ws_floats;
    }
    return mms2ut_gemm_f16(&a, s);
  }
  return linear(c, O, f->wo, f->bo, out, D.Rt, d, d, MMS_EPI_DROP_RESID, textd);
}

extern "C" int mms2ut_gated_fusion_bwd(const mms2ut_gated_fusion* f, const mms2ut_half* dres, int want_dimg,
                                       void* scratch, float* main_ws, int64_t main_ws_floats, float* side_ws,
                                       int64_t side_ws_floats, int side_blocks, hipStream_t main, hipStream_t side) {
  if (int rc = fus_check(f)) return rc;
  MMS_REQUIRE(dres && scratch && f->saved, "gated_fusion_bwd: null gradient / scratch / arena");
  if (!side) side = main;
  const FusDims D = fus_dims(f);
  int64_t sz[FA_N], off[FA_N], ssz[FS_N], so[FS_N];
  fus_arena_sizes(f, D, sz);
  layout(sz, FA_N, off);
  fus_scratch_sizes(f, D, want_dimg, ssz);
  layout(ssz, FS_N, so);
  void* A = f->saved;
  void* S = scratch;
  auto H_ = [&](int slot) { return at<mms2ut_half>(A, off, slot); };
  auto SH = [&](int slot) { return at<mms2ut_half>(S, so, slot); };
  auto SF = [&](int slot) { return at<float>(S, so, slot); };
  const Ctx c{main, side, main_ws, main_ws_floats, side_ws, side_ws_floats, SF(FS_BPART), nullptr, nullptr, false};
  const int64_t d = D.d, Di = D.Di;
  const mms2ut_half* textd = f->p_txt > 0.f ? H_(FA_TEXTD) : f->text;
  const mms2ut_half* imgd = (D.ln_fused || D.extra) ? H_(FA_IMGD) : (!D.ln_fused && (D.pre || f->p_img > 0.f) ? H_(FA_IMGN) : f->img);
  int rc;
  const mms2ut_half *dOp = dres, *dtext = dres;
  int64_t lddop = d, lddtext = d;
  if (D.gate) {
    mms2ut_half *dpre = SH(FS_DPRE), *dmerge = SH(FS_DMERGE);
    if ((rc = mms2ut_gate_bwd(dres, H_(FA_MERGE), H_(FA_G), dpre, dmerge, D.Rt, (int)d, main))) return rc;
    if ((rc = wgrad_auto(c, dpre, d, H_(FA_MERGE), 2 * d, f->g_wg, f->g_bg, D.Rt, d, 2 * d, side_blocks))) return rc;
    if ((rc = dgrad(c, dpre, d, f->wg, f->wt_g, dmerge, D.Rt, d, 2 * d, MMS_EPI_F16_ACC))) return rc;
    dOp = dmerge; lddop = 2 * d;
    dtext = dmerge + d; lddtext = 2 * d;
  }
  if ((rc = wgrad_auto(c, dOp, lddop, H_(FA_O), d, f->g_wo, f->g_bo, D.Rt, d, d, side_blocks))) return rc;
  mms2ut_half* dO = SH(FS_DO);
  if ((rc = dgrad(c, dOp, lddop, f->wo, f->wt_o, dO, D.Rt, d, d))) return rc;
  // attention backward (model.attn_bwd)
  const float scale = (float)pow((double)d, -0.5);
  const mms2ut_half *q = H_(FA_Q), *kv = H_(FA_KV), *P = H_(FA_P), *Pd = f->p_attn > 0.f ? H_(FA_PD) : P;
  mms2ut_half *dq = SH(FS_DQ), *dkv = SH(FS_DKV), *dPd = SH(FS_DPD);
  const int B = (int)D.B, Te = (int)D.Te, Tk = (int)D.Tk;
  const int64_t sS = D.Te * D.ldS;
  {
    mms2ut_gemm_args a = batched(dO, kv + d, dPd, Te, Tk, (int)d, 1, 1, d, 2 * d, D.ldS, B, D.Te * d, D.Tk * 2 * d, sS, 1.f);
    if ((rc = mms2ut_gemm_f16(&a, main))) return rc;
    a = batched(Pd, dO, dkv + d, Tk, (int)d, Te, 0, 0, D.ldS, d, 2 * d, B, sS, D.Te * d, D.Tk * 2 * d, 1.f);
    if ((rc = mms2ut_gemm_f16(&a, main))) return rc;
  }
  if ((rc = mms2ut_attn_softmax_bwd(P, dPd, dPd, B, 1, Te, Tk, D.ldS, nullptr, 0, 0, f->p_attn,
                                    f->p_attn > 0.f ? f->seed : 0, f->p_attn > 0.f ? f->off_attn : 0, main))) return rc;
  {
    mms2ut_gemm_args a = batched(dPd, kv, dq, Te, (int)d, Tk, 1, 0, D.ldS, 2 * d, d, B, sS, D.Tk * 2 * d, D.Te * d, scale);
    if ((rc = mms2ut_gemm_f16(&a, main))) return rc;
    a = batched(dPd, q, dkv, Tk, (int)d, Te, 0, 0, D.ldS, d, 2 * d, B, sS, D.Te * d, D.Tk * 2 * d, scale);
    if ((rc = mms2ut_gemm_f16(&a, main))) return rc;
  }
  if (D.extra) {
    // bias_k / bias_v gradients: the batch sum of the extra key row's gradient (main stream), then
    // that row is zeroed for the k|v weight gradient
    mms2ut_half* rows = dkv + D.Ti * 2 * d;
    const int np = mms2ut_colsum_nparts(D.B);
    if ((rc = mms2ut_colsum_f16(rows, D.B, (int)(2 * d), D.Tk * 2 * d, SF(FS_KVP), np, main))) return rc;
    if ((rc = mms2ut_colsum_parts(SF(FS_KVP), np, (int)(2 * d), f->g_bias_kv, 0, main))) return rc;
    if ((rc = zero_rows(rows, D.Tk * 2 * d, 2 * d, D.B, main))) return rc;
  }
  if ((rc = wgrad_auto(c, dkv, 2 * d, imgd, Di, f->g_wkv, f->g_bkv, D.Rk, 2 * d, Di, side_blocks))) return rc;
  if (D.ln_fused) {
    mms2ut_half* dimgd = SH(FS_DIMGD);
    if ((rc = dgrad(c, dkv, 2 * d, f->wkv, f->wt_kv, dimgd, D.Rk, 2 * d, Di))) return rc;
    if ((rc = mms2ut_layernorm_bwd_ex(dimgd, f->img, f->ln_g, at<float>(A, off, FA_IM), at<float>(A, off, FA_IR), nullptr,
                                      want_dimg ? SH(FS_DIMGIN) : nullptr, SF(FS_LNP), D.Ri, (int)Di, nullptr, 0.f, 0, 0,
                                      D.extra ? D.Ti : 0, D.extra ? D.Tk : 0, f->p_img, f->p_img > 0.f ? f->seed : 0,
                                      f->p_img > 0.f ? f->off_img : 0, main))) return rc;
    if ((rc = fork(c)) ||
        (rc = mms2ut_colsum_parts(SF(FS_LNP), mms2ut_layernorm_bwd_nparts(D.Ri, (int)Di), (int)(2 * Di), f->g_ln, 0, side)))
      return rc;
  } else if (D.pre || want_dimg) {
    mms2ut_half* dimgd = SH(FS_DIMGD);
    if ((rc = dgrad(c, dkv, 2 * d, f->wkv, f->wt_kv, dimgd, D.Rk, 2 * d, Di))) return rc;
    mms2ut_half* dimg = dimgd;
    if (D.extra) {
      dimg = SH(FS_DIMG);
      if ((rc = mms2ut_copy2d(dimgd, D.Tk * Di, dimg, D.Ti * Di, D.B, (int)(D.Ti * Di), main))) return rc;
    }
    if (f->p_img > 0.f && (rc = mms2ut_dropout_fwd(dimg, dimg, D.Ri * Di, f->p_img, f->seed, f->off_img, main))) return rc;
    if (D.pre) {
      if ((rc = ln_bwd(c, dimg, f->img, f->ln_g, at<float>(A, off, FA_IM), at<float>(A, off, FA_IR), nullptr,
                       want_dimg ? SH(FS_DIMGIN) : nullptr, nullptr, 0.f, 0, 0, SF(FS_LNP), f->g_ln, D.Ri, (int)Di)))
        return rc;
    }
  }
  if ((rc = wgrad_auto(c, dq, d, textd, d, f->g_wq, f->g_bq, D.Rt, d, d, side_blocks))) return rc;
  mms2ut_half* dtt = SH(FS_DTEXT);
  if ((rc = mms2ut_copy2d(dtext, lddtext, dtt, d, D.Rt, (int)d, main))) return rc;
  if ((rc = dgrad(c, dq, d, f->wq, f->wt_q, dtt, D.Rt, d, d, MMS_EPI_F16_ACC))) return rc;
  if (f->p_txt > 0.f && (rc = mms2ut_dropout_fwd(dtt, dtt, D.Rt * d, f->p_txt, f->seed, f->off_txt, main))) return rc;
  return 0;
}

extern "C" int mms2ut_workspace_size(int op, const void* desc, int64_t* sizes) {
  MMS_REQUIRE(desc && sizes, "workspace_size: null");
  int rc;
  switch (op) {
    case MMS_OP_LAYER: {
      const mms2ut_layer* L = static_cast<const mms2ut_layer*>(desc);
      if ((rc = mms2ut_layer_arena(L, nullptr, &sizes[0])) || (rc = mms2ut_layer_scratch(L, 0.f, nullptr, &sizes[1])))
        return rc;
      return mms2ut_layer_ws(L, &sizes[2], &sizes[3]);
    }
    case MMS_OP_CONV1D_GLU: {
      const mms2ut_conv1d_glu* c = static_cast<const mms2ut_conv1d_glu*>(desc);
      if ((rc = mms2ut_conv1d_glu_arena(c, nullptr, &sizes[0])) || (rc = mms2ut_conv1d_glu_scratch(c, nullptr, &sizes[1])))
        return rc;
      return mms2ut_conv1d_glu_ws(c, &sizes[2], &sizes[3]);
    }
    case MMS_OP_GATED_FUSION: {
      const mms2ut_gated_fusion* f = static_cast<const mms2ut_gated_fusion*>(desc);
      if ((rc = mms2ut_gated_fusion_arena(f, nullptr, &sizes[0])) ||
          (rc = mms2ut_gated_fusion_scratch(f, 0, nullptr, &sizes[1])))
        return rc;
      return mms2ut_gated_fusion_ws(f, &sizes[2], &sizes[3]);
    }
    default:
      mms::set_error("workspace_size: unknown op %d", op);
      return 1;
  }
}
