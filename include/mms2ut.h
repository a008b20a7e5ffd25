/*
 * libmms2ut_hip — C-ABI of the MI355X-native mm_s2ut_transformer training path.
 *
 * Every entry point takes raw device pointers, int64 sizes/strides, scalars and the HIP stream to
 * enqueue on (PyTorch's current stream).  All buffers, including workspaces, belong to the caller
 * (PyTorch's caching allocator).  The library keeps one piece of state: a per-device pool of
 * zeroed ticket arrays for the short-M GEMM's in-kernel split-K (4 MiB, allocated on the device's
 * first such launch; one 8 KiB slice per (device, stream), handed out under a mutex; every completed
 * launch leaves its slice zero).  Apart from that pool, the GEMM route switches below and the bound
 * step seed, entry points keep no state and may be called from several host threads; kernels are
 * only ever enqueued on the passed stream.  Functions return 0 on success and non-zero on error;
 * mms2ut_last_error() returns the message (thread-local).
 *
 * Each entry cites the reference interface (or the fairseq/PyTorch op it executes for the
 * reference) that it replaces — see SURVEY.md §8(a)/(b) and INTEGRATION.md.
 */
#ifndef MMS2UT_H
#define MMS2UT_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef _Float16 mms2ut_half;

/* ---------------------------------------------------------------- errors / introspection */
const char* mms2ut_last_error(void);
/* A non-blocking HIP stream (hipStreamNonBlocking) at a priority clamped to the device's range
 * (lower = more urgent): the trainer's critical-path and weight-gradient side streams, so that no
 * work a caller leaves on the legacy NULL stream implicitly orders itself behind them.           */
int mms2ut_stream_create(int priority, hipStream_t* out);
/* Destroys a stream from mms2ut_stream_create (after the work enqueued on it has completed).     */
int mms2ut_stream_destroy(hipStream_t stream);
int mms2ut_version(void);

/* ---------------------------------------------------------------- GEMM (MFMA fp16, fp32 acc)
 * Replaces every nn.Linear / bmm / conv-as-GEMM the reference executes through cuBLAS:
 * fairseq MultiheadAttention q/k/v/out_proj, TransformerEncoderLayer/DecoderLayer fc1/fc2,
 * Conv1dSubsampler convs (im2col), fusion projections (fuse.py:76-78,116; nn.MultiheadAttention
 * in_proj/out_proj for fuse.py:161), the gate dense (mm_s2s_transformer.py:613-614) and the tied
 * output projection — forward, dgrad and wgrad.
 *   C[m][n] = epi(alpha * sum_k A(m,k) B(n,k))
 *   A(m,k) = a_kcontig ? A[m*lda+k] : A[k*lda+m];  B(n,k) = b_kcontig ? B[n*ldb+k] : B[k*ldb+n]
 *   batch z in [0,batch): z1 = z / bdiv, z2 = z % bdiv; X += z1*sX1 + z2*sX2 (elements)
 *   split-K (epi = MMS_EPI_F32 only): slab s written at C + s*sCsplit (fp32)            */
enum {
  MMS_EPI_F16 = 0,          /* C = alpha*acc (+bias)                                      */
  MMS_EPI_RELU_DROP = 1,    /* C = dropout(relu(alpha*acc + bias))        (fc1)           */
  MMS_EPI_DROP_RESID = 2,   /* C = aux + dropout(alpha*acc + bias)        (out_proj, fc2) */
  MMS_EPI_F32 = 3,          /* C(fp32) = alpha*acc                        (split-K slabs) */
  MMS_EPI_GATE = 4,         /* g = sigmoid(acc+bias); C = t + g*(o-t); out2 = g; o = aux[:, :N], t = aux[:, N:2N] */
  MMS_EPI_RELU_DROP_BWD = 5,/* C = aux>0 ? alpha*acc/(1-p) : 0            (fc2 dgrad -> fc1 pre-act) */
  MMS_EPI_F16_ACC = 6,      /* C += alpha*acc                                               */
  MMS_EPI_GELU_DROP = 7,    /* z = alpha*acc + bias; out2 = z; C = dropout(gelu(z))  (torch F.gelu, erf form) */
  MMS_EPI_GELU_DROP_BWD = 8 /* z = aux: C = keep ? alpha*acc/(1-p) * gelu'(z) : 0 (mask regenerated from seed/offset) */
};

typedef struct mms2ut_gemm_args {
  const mms2ut_half* A;
  const mms2ut_half* B;
  void* C;
  int M, N, K;
  int a_kcontig, b_kcontig;
  int64_t lda, ldb, ldc;
  int batch, bdiv;
  int64_t sA1, sA2, sB1, sB2, sC1, sC2;
  int splitk;
  int64_t sCsplit;
  int epi;
  float alpha;
  const mms2ut_half* bias;
  const mms2ut_half* aux;
  int64_t ldaux, sX1, sX2;
  mms2ut_half* out2;
  int64_t ldo2;
  float dropout_p;
  uint64_t seed, offset;
  int64_t ld_rng;
  /* optional (epi = MMS_EPI_F32, a_kcontig = 0): fp32 A-row sums alpha*sum_k A(m,k) of split s
   * -> rowsum[s*ld_rowsum + m].  The weight-gradient GEMM's A is dy^T, so these are the split-K
   * partials of the bias gradient (replaces a separate column-sum pass over dy).             */
  float* rowsum;
  int64_t ld_rowsum;
  /* split-K with a fused-epilogue fixup (any epi but MMS_EPI_F32, batch 1, splitk > 1, N % 4 == 0):
   * the splits write alpha-scaled fp32 partials to splitk_ws[s][M][N] (>= splitk*M*N floats),
   * then one pass sums them in split order and applies the epilogue exactly as the unsplit GEMM
   * (same bias / residual / dropout counters).  For the short-M shapes (decoder tokens) whose
   * unsplit grid covers a tenth of the CUs.                                                       */
  float* splitk_ws;
  int64_t splitk_ws_floats;
} mms2ut_gemm_args;

int mms2ut_gemm_f16(const mms2ut_gemm_args* args, hipStream_t stream);
/* NT shapes (both operands K-contiguous, batch 1, no split) may run on 96 / 160 / 192 x 128 tiles
 * instead of 128 x 128 ones when that takes fewer rounds of the 512 block slots, or (96 rows) fills
 * a short single round better, weighted by each height's measured per-round cost (e.g. M = 11-16 k
 * rows x N = 768: one round instead of two); bit-identical results.  mode 1: by that rule (default;
 * env MMS2UT_GEMM_TALL overrides it at first use), 0: never, 2 / 3 / 5: 160 / 192 / 96-row tiles
 * for every qualifying NT shape (tests).                                                          */
int mms2ut_gemm_set_tall(int mode);

/* Short-M NT GEMMs (a 128x128 grid of fewer than 128 tiles: the decoder's ~470-row projections).
 * mode 1 (default; env MMS2UT_GEMM_SKINNY overrides it at first use): a measured route table —
 * N <= 1024 on the short-M kernel (one-shot operand loads per small tile, K split across blocks
 * with an in-kernel last-arrival reduction into the caller's splitk_ws, epilogue fused, no second
 * launch), N > 1024 with K <= 1024 unsplit on the 128-row tiles, the rest on the split-K + fixup
 * route the caller asked for; 0: always the caller's route (A/B runs, tests); 2: the short-M kernel
 * for every short-M shape (tests).                                                              */
int mms2ut_gemm_set_skinny(int mode);
/* Test hook of the short-M kernel's split-K hand-off (placement-independent: write-through partials,
 * a relaxed agent-scope ticket, write-through reads).  scatter != 0 deals the splits of every tile
 * over different XCD groups (bid % 8) instead of keeping them together; xcc_out (device, >= grid
 * ints, or NULL) receives each block's hardware XCD id (HW_REG_XCC_ID).  Bits are identical either
 * way.                                                                                         */
int mms2ut_gemm_skinny_debug(int scatter, int* xcc_out);
/* Test hook of the fused epilogues: staged != 0 routes every fp16 epilogue through the fp32 LDS
 * staging (the round-5 form) instead of the register epilogue (plain / ReLU-dropout: element math
 * in the MFMA layout, fp16 through LDS).  Bits are identical either way.                        */
int mms2ut_gemm_set_epilogue(int staged);

/* Grouped weight gradients of one transformer layer (torch.nn.Linear weight / bias grads of the
 * reference layer's projections): for each of the n <= 8 problems, dW[N, K] = dy[rows, N]^T @
 * x[rows, K] (fp16, row stride K, overwritten) and, when db != NULL, db[N] = column sums of dy —
 * all in ONE launch over the union of the problems' 128x128 tiles, unsplit (fp32 accumulation over
 * all rows, no split-K slabs).  lddy, ldx multiples of 8; N, K multiples of 8; dy, x, dW 16-B
 * aligned.  Deterministic (fixed reduction order per tile).  max_blocks > 0 caps the grid
 * (rounded down to a multiple of 8): blocks then walk the tiles persistently, so a launch on a
 * side stream never holds more than that many block slots (0: one block per tile).            */
typedef struct mms2ut_wgrad {
  const mms2ut_half* dy;
  int64_t lddy;
  const mms2ut_half* x;
  int64_t ldx;
  mms2ut_half* dW;
  mms2ut_half* db;
  int N, K;
} mms2ut_wgrad;
int mms2ut_wgrad_group(const mms2ut_wgrad* w, int n, int64_t rows, int max_blocks, hipStream_t stream);

/* live GEMM timing for the benchmark roofline: between begin/end every mms2ut_gemm_f16 launch
 * is bracketed by HIP events on its own stream (or, in stamp mode below, timed by its own
 * workgroups); end() synchronises and returns the summed event time (0 in stamp mode), the launch
 * count and the launched (padded) FLOPs.  Bench-only instrumentation, not thread-safe.      */
int mms2ut_profile_begin(int max_launches);
int mms2ut_profile_end(float* total_ms, int* launches, double* flops);
/* algorithmic HBM bytes of the GEMM launches of the last begin/end window (A and B read once, C
 * written once; fp32 split-K slabs, residual / accumulate / gate operands included)            */
int mms2ut_profile_bytes(double* bytes);
/* per-launch record of the last finished window (first n launches): kernel ms, launched FLOPs and
 * a class word: bit0 A K-contiguous, bit1 B K-contiguous, bits 2-7 epilogue, bit8 batched,
 * bit9 split-K.  Lets the bench split forward / dgrad (NT) from weight-gradient (TN) launches.   */
int mms2ut_profile_launches(float* ms, double* flops, int* cls, int n);
/* the same window's shapes: mnk[4i..4i+3] = M, N, K, batch * splitk of launch i                  */
int mms2ut_profile_shapes(int* mnk, int n);
/* stamp mode for the open window (call right after profile_begin): instead of events, every GEMM
 * kernel's blocks store {start, end} s_memrealtime ticks (2 x u64 per block) into `stamps`
 * (device, 16-B aligned, room for cap_blocks blocks).  profile_blocks then gives, per launch,
 * the first block slot and one past the last (a split-K fixup's blocks follow its GEMM's; a
 * value > cap_blocks means the buffer overflowed and the launch was not recorded).  A launch's
 * duration = max(end) - min(start) over its slots, in ticks of mms2ut_wallclock_khz.  Bench-only
 * instrumentation (no reference counterpart).                                                    */
int mms2ut_profile_stamps(unsigned long long* stamps, long cap_blocks);
int mms2ut_profile_blocks(long* first_last, int n);
int mms2ut_wallclock_khz(int* khz);

/* sum `nsplit` fp32 slabs [rows, cols] (slab stride `slab`) * alpha -> out, row stride ldo.
 * mode bit0: fp16 output (else fp32); bit1: accumulate into out (else overwrite)            */
int mms2ut_splitk_reduce(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                         void* out, int64_t ldo, int mode, float alpha, hipStream_t stream);
/* the weight-gradient epilogue in one launch: fp16 dW = sum of `nsplit` fp32 slabs [rows, cols]
 * (row stride ldo) and fp16 db[rows] = sum of the GEMM's rowsum partials rs_slabs[nsplit][rows].
 * rows, cols, ldo multiples of 4.  Replaces the bias column-sum of dy (fairseq Linear.bias.grad). */
int mms2ut_splitk_reduce_bias(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                              mms2ut_half* out, int64_t ldo, const float* rs_slabs,
                              mms2ut_half* rs_out, hipStream_t stream);

/* batched transpose of row-major fp16 matrices: dst[d.dst + c*rows + r] = src[d.src + r*cols + c]
 * (element offsets).  descs (DEVICE memory) sorted by tile0, the first 64x64 tile of each matrix;
 * rows, cols multiples of 8.  Keeps the W^T images that make every dgrad GEMM NT (K-contiguous
 * operands) — the reference's cuBLAS dgrad reads W in place.                                    */
typedef struct mms2ut_transpose_desc {
  int64_t src, dst;
  int32_t rows, cols, tile0, pad;
} mms2ut_transpose_desc;
int mms2ut_transpose_batch(const mms2ut_half* src, mms2ut_half* dst, const mms2ut_transpose_desc* descs,
                           int n, int total_tiles, hipStream_t stream);

/* `waiter` waits for all work enqueued on `signaler` so far (event record + stream wait).
 * Forks/joins the weight-gradient side stream (the reference's DDP/autograd stream overlap). */
int mms2ut_stream_wait(hipStream_t waiter, hipStream_t signaler);
/* Device-scope events (no timing, no system-scope fence): ordering between this process's streams
 * on one GPU — the deferred optimizer chunks before the next forward reads them, the weight
 * transpose before the dgrad GEMMs, per-group gradient hand-offs (torch's CUDA events in the
 * reference's DDP / autograd stream syncs).  Not for host synchronisation.                       */
int mms2ut_event_create(hipEvent_t* out);
int mms2ut_event_record(hipEvent_t event, hipStream_t stream);
int mms2ut_event_wait(hipStream_t stream, hipEvent_t event);
int mms2ut_event_destroy(hipEvent_t event);
/* HIP-graph replay of the training step: every dropout kernel adds *delta (a device uint64) to
 * the seed it was launched or captured with; delta == NULL (the default) leaves seeds unchanged.
 * mms2ut_step_seed_advance(delta, inc) is the first node of a captured step (delta += inc), so
 * each replay draws fresh masks (fairseq reseeds torch's generator per update in
 * Trainer.train_step; here the per-update seed lives on the device).                           */
int mms2ut_bind_step_seed(const uint64_t* delta);
int mms2ut_step_seed_advance(uint64_t* delta, uint64_t inc, hipStream_t stream);

/* ---------------------------------------------------------------- LayerNorm (eps, affine)
 * Replaces fairseq LayerNorm (self_attn_layer_norm / final_layer_norm / encoder_attn_layer_norm /
 * encoder.layer_norm / decoder.layer_norm) and nn.LayerNorm image_pre_norm_module
 * (mm_s2s_transformer.py:188-190,595).  Rows of D fp16, statistics fp32.                  */
int mms2ut_layernorm_fwd(const mms2ut_half* x, const mms2ut_half* gamma, const mms2ut_half* beta,
                         mms2ut_half* y, float* mean, float* rstd, int64_t rows, int D, float eps,
                         hipStream_t stream);
/* dx = LN'(dy) (+ dres if non-null); partial dgamma/dbeta sums -> part[nblk][2][D] (fp32).
 * dx may be null (parameter grads only).  If dxd is non-null it also receives dropout(dx) with
 * counters offset + row*D + col: the residual-branch dropout of the sublayer below, whose
 * output-projection gradient consumes it (saves a separate dropout pass).                  */
int mms2ut_layernorm_bwd(const mms2ut_half* dy, const mms2ut_half* x, const mms2ut_half* gamma,
                         const float* mean, const float* rstd, const mms2ut_half* dres,
                         mms2ut_half* dx, float* part, int64_t rows, int D, mms2ut_half* dxd,
                         float p, uint64_t seed, uint64_t offset, hipStream_t stream);
int mms2ut_layernorm_bwd_parts(int64_t rows);
/* number of [2*D] fp32 partial rows mms2ut_layernorm_bwd{,_ex} write for (rows, D) */
int mms2ut_layernorm_bwd_nparts(int64_t rows, int D);
/* layernorm_fwd with an output layout and dropout folded in (the fusion image path,
 * mm_s2s_transformer.py:188-190 image_pre_norm -> SA_image_dropout -> [B, Ti(+1), Di] keys):
 * input row r is written to output row (r / grp) * grp_out + r % grp (grp = 0: identity), and
 * y = dropout_p(LN(x)) with counters offset + r*D + col (the unpadded element index).         */
int mms2ut_layernorm_fwd_ex(const mms2ut_half* x, const mms2ut_half* gamma, const mms2ut_half* beta,
                            mms2ut_half* y, float* mean, float* rstd, int64_t rows, int D, float eps,
                            int64_t grp, int64_t grp_out, float p, uint64_t seed, uint64_t offset,
                            hipStream_t stream);
/* layernorm_bwd whose dy is read through the same layout (row r from (r / dy_grp) * dy_grp_out +
 * r % dy_grp) and dropout (dy_p, dy_seed, dy_offset; unpadded counters): the backward of
 * layernorm_fwd_ex without materialising the unpadded, dropped-out gradient.  D % 256 == 0.    */
int mms2ut_layernorm_bwd_ex(const mms2ut_half* dy, const mms2ut_half* x, const mms2ut_half* gamma,
                            const float* mean, const float* rstd, const mms2ut_half* dres,
                            mms2ut_half* dx, float* part, int64_t rows, int D, mms2ut_half* dxd,
                            float p, uint64_t seed, uint64_t offset, int64_t dy_grp, int64_t dy_grp_out,
                            float dy_p, uint64_t dy_seed, uint64_t dy_offset, hipStream_t stream);
/* column sums of fp32 partials [nparts][ncol] -> out (fp16), out += if accumulate */
int mms2ut_colsum_parts(const float* part, int nparts, int ncol, mms2ut_half* out, int accumulate,
                        hipStream_t stream);
/* column sums of an fp16 matrix [rows][cols] (row stride ld) -> part[nparts][cols] fp32 (bias grads) */
int mms2ut_colsum_f16(const mms2ut_half* x, int64_t rows, int cols, int64_t ld, float* part,
                      int nparts, hipStream_t stream);
int mms2ut_colsum_nparts(int64_t rows);

/* ---------------------------------------------------------------- attention softmax
 * Masked softmax over attention scores S[z][Tq][ldS] (fp16) with per-batch key lengths
 * (key padding mask, fairseq/torch MHA key_padding_mask), optional causal mask
 * (buffered_future_mask), optional "always-valid" trailing key (add_bias_kv column of
 * nn.MultiheadAttention, fuse.py:161), and attention-prob dropout (p, counter RNG).
 * Keys may instead be masked by key_mask[b*ld_mask + j] != 0 (bool key_padding_mask).
 * Writes P (undropped) and Pd (dropped, may alias P when p == 0).  z = b*H + h.            */
int mms2ut_attn_softmax_fwd(const mms2ut_half* S, mms2ut_half* P, mms2ut_half* Pd, int Z, int H,
                            int Tq, int Tk, int64_t ldS, const int32_t* key_len,
                            const uint8_t* key_mask, int64_t ld_mask, int causal,
                            int extra_key, float p, uint64_t seed, uint64_t offset,
                            hipStream_t stream);
/* dS = P * (dPd*mask/(1-p) - sum_j Pd_j dPd_j) ; dP may alias dS                            */
int mms2ut_attn_softmax_bwd(const mms2ut_half* P, const mms2ut_half* dPd, mms2ut_half* dS, int Z,
                            int H, int Tq, int Tk, int64_t ldS, const int32_t* key_len, int causal,
                            int extra_key, float p, uint64_t seed, uint64_t offset,
                            hipStream_t stream);

/* ---------------------------------------------------------------- fused multi-head attention
 * Flash-style fwd/bwd (scores stay on chip) for fairseq MultiheadAttention in the encoder
 * (self, key padding), decoder (causal self + target padding) and decoder cross attention
 * (encoder padding): softmax(scale * q k^T + masks) -> dropout(p) -> @ v, per (b, h).
 * Element (b, h, t, d) of X lives at X[b*sXb + t*ldX + h*hd + d] (sXb = 0 -> T*ldX).
 * Padding: keys j >= key_len[b] masked (key_len may be null).  head_dim in {64, 96, 128}.
 * lse[z*Tq + t] (z = b*H + h) receives the row log-sum-exp for the backward pass.          */
typedef struct mms2ut_attn_args {
  const mms2ut_half* q;
  const mms2ut_half* k;
  const mms2ut_half* v;
  mms2ut_half* o;
  int64_t ldq, ldk, ldv, ldo;
  int64_t sqb, skb, svb, sob;
  int B, H, Tq, Tk, hd;
  const int32_t* key_len;
  int causal;
  float scale;
  float p;
  uint64_t seed, offset;
  float* lse;
} mms2ut_attn_args;

int mms2ut_mha_varlen_fwd(const mms2ut_attn_args* args, hipStream_t stream);
/* dq/dk/dv written (not accumulated); Dd: fp32 workspace [B*H*Tq]                          */
int mms2ut_mha_varlen_bwd(const mms2ut_attn_args* args, const mms2ut_half* dout, int64_t lddo,
                          int64_t sdob, float* Dd, mms2ut_half* dq, int64_t lddq, int64_t sdqb,
                          mms2ut_half* dk, int64_t lddk, int64_t sdkb, mms2ut_half* dv,
                          int64_t lddv, int64_t sdvb, hipStream_t stream);

/* ---------------------------------------------------------------- elementwise / embedding */
/* y = dropout(x) elementwise (n elements, counter offset) ; y may alias x                   */
int mms2ut_dropout_fwd(const mms2ut_half* x, mms2ut_half* y, int64_t n, float p, uint64_t seed,
                       uint64_t offset, hipStream_t stream);
/* materialise the keep-mask (uint8) the kernels use — for parity tests / debugging          */
int mms2ut_dropout_mask(uint8_t* keep, int64_t n, float p, uint64_t seed, uint64_t offset,
                        hipStream_t stream);
/* encoder input: x[b,t,:] = dropout(scale*h[b,t,:] + pos[t+2 if t<len[b] else 1, :])
 * (fairseq S2TTransformerEncoder._forward: embed_scale, SinusoidalPositionalEmbedding(pad mask)) */
int mms2ut_encoder_embed_fwd(const mms2ut_half* h, const mms2ut_half* pos_table, const int32_t* len,
                             mms2ut_half* x, int B, int T, int D, float scale, float p,
                             uint64_t seed, uint64_t offset, hipStream_t stream);
/* backward of the above w.r.t. h: dh = scale * dropout_mask * dx                             */
int mms2ut_scale_dropout_bwd(const mms2ut_half* dx, mms2ut_half* dh, int64_t n, float scale,
                             float p, uint64_t seed, uint64_t offset, hipStream_t stream);
/* decoder input (fairseq TransformerDecoder.extract_features, StackedEmbedding n=1):
 * x = dropout(scale*E[tok] + pos[make_positions(tok)])                                      */
int mms2ut_token_embed_fwd(const int64_t* tok, const mms2ut_half* E, const mms2ut_half* pos_table,
                           mms2ut_half* x, int B, int T, int D, int pad_idx, float scale, float p,
                           uint64_t seed, uint64_t offset, hipStream_t stream);
/* dE[tok] += scale*mask*dx (fp32 accumulation buffer dE32 [V][D], D <= 1024; pad rows skipped).
 * Deterministic: one block per vocabulary row sums its positions in ascending order (no float
 * atomics), so the tied-embedding gradient is bit-reproducible.  Every block scans all B*T token
 * ids (O(V * B*T) id reads, ~0.05 ms at the unit vocabulary V = 1004): sized for unit / character
 * vocabularies, not for 10^4+ word vocabularies.                                              */
int mms2ut_token_embed_bwd(const int64_t* tok, const mms2ut_half* dx, float* dE32, int B, int T,
                           int D, int V, int pad_idx, float scale, float p, uint64_t seed,
                           uint64_t offset, hipStream_t stream);
/* out(fp16) = a(fp16) + b32(fp32) elementwise                                                */
int mms2ut_add_f32_to_f16(const mms2ut_half* a, const float* b, mms2ut_half* out, int64_t n,
                          hipStream_t stream);
/* GLU over the channel (last) dim: y[r, c] = x[r, c] * sigmoid(x[r, c + C]), x row stride 2C */
int mms2ut_glu_fwd(const mms2ut_half* x, mms2ut_half* y, int64_t rows, int C, hipStream_t stream);
int mms2ut_glu_bwd(const mms2ut_half* x, const mms2ut_half* dy, mms2ut_half* dx, int64_t rows,
                   int C, hipStream_t stream);
/* Conv1d (stride 2, pad k/2) as implicit GEMM: im2col of x[B][Tin][C] -> col[B*Tout][C*k]
 * ordered (c, k) to match the PyTorch weight [out][C][k] (fairseq Conv1dSubsampler)          */
int mms2ut_im2col(const mms2ut_half* x, mms2ut_half* col, int B, int Tin, int Tout, int C, int k,
                  int stride, int pad, hipStream_t stream);
/* im2col with a row stride ldcol >= C*k; columns [C*k, ldcol) are zero (K padded to whole GEMM
 * k-tiles: the first conv's C*k = 80*5 = 400 -> 448)                                          */
int mms2ut_im2col_ld(const mms2ut_half* x, mms2ut_half* col, int B, int Tin, int Tout, int C, int k,
                     int stride, int pad, int ldcol, hipStream_t stream);
int mms2ut_col2im(const mms2ut_half* dcol, mms2ut_half* dx, int B, int Tin, int Tout, int C, int k,
                  int stride, int pad, hipStream_t stream);
/* fusion gate backward (mm_s2s_transformer.py:613-618):
 * dpre = dres*(o-t)*g*(1-g); dmerge_direct = [dres*g, dres*(1-g)]                            */
int mms2ut_gate_bwd(const mms2ut_half* dres, const mms2ut_half* merge, const mms2ut_half* g,
                    mms2ut_half* dpre, mms2ut_half* dmerge, int64_t rows, int D,
                    hipStream_t stream);
/* copy rows with strides (cols fp16 elements)                                               */
int mms2ut_copy2d(const mms2ut_half* src, int64_t lds, mms2ut_half* dst, int64_t ldd, int64_t rows,
                  int cols, hipStream_t stream);
/* copy2d, and columns [cols, cols + zcols) of every dst row set to zero in the same launch
 * (src may be NULL with cols = 0: a strided zero fill) — the zero-padded weight / key layouts of
 * the subsampler and the fusion without a separate memset                                     */
int mms2ut_copy2d_pad(const mms2ut_half* src, int64_t lds, mms2ut_half* dst, int64_t ldd, int64_t rows,
                      int cols, int zcols, hipStream_t stream);
/* out = a + b (fp16) */
int mms2ut_add_f16(const mms2ut_half* a, const mms2ut_half* b, mms2ut_half* out, int64_t n,
                   hipStream_t stream);

/* ---------------------------------------------------------------- label-smoothed CE
 * fairseq speech_to_unit -> LabelSmoothedCrossEntropyCriterion.compute_loss (reference copy
 * criterions/speech_to_speech_criterion.py:58-102): fp32 log_softmax over V, eps-smoothing,
 * pad targets ignored, reduce=sum.  loss_out[2] += {loss, nll} (fp32; per-block partials in
 * part[2 * MMS_LS_XENT_PARTS] summed in a fixed order: bit-reproducible).  lse[rows] saved for
 * the backward.                                                                              */
#define MMS_LS_XENT_PARTS 512
int mms2ut_ls_xent_fwd(const mms2ut_half* logits, int64_t ld, const int64_t* target, int64_t rows,
                       int V, float eps, int pad_idx, float* lse, float* part, float* loss_out,
                       hipStream_t stream);
/* the same, for a trainer's step log: acc[0..1] += {loss, nll} (may be NULL) and call_out[0..1] =
 * this call's {loss, nll} (written, may be NULL) — no zeroed accumulator and no copies        */
int mms2ut_ls_xent_fwd_log(const mms2ut_half* logits, int64_t ld, const int64_t* target, int64_t rows,
                           int V, float eps, int pad_idx, float* lse, float* part, float* acc, float* call_out,
                           hipStream_t stream);
/* dlogits = grad * ((1-eps-eps_i)(p - onehot) + eps_i(V p - 1)), 0 on pad rows; in place OK */
int mms2ut_ls_xent_bwd(const mms2ut_half* logits, int64_t ld, const int64_t* target, int64_t rows,
                       int V, float eps, int pad_idx, const float* lse, const float* grad,
                       mms2ut_half* dlogits, hipStream_t stream);

/* ---------------------------------------------------------------- FP16Optimizer + Adam
 * fairseq FP16Optimizer (fp32 master, dynamic loss scale) + clip_grad_norm_ + Adam (fairseq
 * optim/adam.py) + DynamicLossScaler, entirely device-side (no host sync per step).
 * `ost` is a device fp32 state vector (indices MMS_OST_*), initialised by the host once
 * (loss_scale = --fp16-init-scale, iter = 0, last_overflow = -1, step = 0).
 *   grad_sqnorm -> grad_norm_finalize (mult = 1/(loss_scale*sample_size), norm, overflow)
 *   -> optim_prepare (Adam step/step size, clip coef, scaler update) -> adam (skips on overflow) */
enum {
  MMS_OST_MULT = 0, MMS_OST_GNORM = 1, MMS_OST_OVERFLOW = 2, MMS_OST_STEP = 3,
  MMS_OST_STEP_SIZE = 4, MMS_OST_LOSS_SCALE = 5, MMS_OST_ITER = 6, MMS_OST_LAST_OVERFLOW = 7,
  MMS_OST_LAST_RESCALE = 8, MMS_OST_CLIP_COEF = 9, MMS_OST_FATAL = 10, MMS_OST_LR = 11,
  MMS_OST_INCONSISTENT = 12, MMS_OST_SIZE = 16
};
int mms2ut_grad_sqnorm(const mms2ut_half* grad, int64_t n, float* part, int nparts,
                       hipStream_t stream);
int mms2ut_grad_norm_finalize(const float* part, int nparts, float* ost, const float* sample_size,
                              hipStream_t stream);
/* lr = fairseq inverse_sqrt(lr, warmup_init_lr, warmup_updates) evaluated on device at the count of
 * completed (non-overflow) updates, stored in ost[MMS_OST_LR] for adam. */
int mms2ut_optim_prepare(float* ost, float lr, float warmup_init_lr, float warmup_updates, float beta1,
                         float beta2, float clip_norm, float scale_window, float min_loss_scale,
                         hipStream_t stream);
/* CTC loss of a multitask CTC head (fairseq CtcCriterion: F.ctc_loss on log_softmax(logits.float()),
 * reduction "sum").  logits: fp16 batch-major rows b*T + t, leading dim ld >= V; targets int64
 * [B, tgt_ld] (first tgt_len[b] used, max_tgt_len = max tgt_len); in_len / tgt_len int32 [B];
 * work: fp32 scratch of mms2ut_ctc_workspace_floats(B, T, max_tgt_len) elements, kept from fwd to
 * bwd.  fwd ADDS the summed loss to *loss_sum (zero_infinity: infinite per-utterance losses count
 * 0).  bwd writes dlogits (ldd >= V, padded rows/columns 0) = grad_scale[0] * d loss / d logits;
 * impossible alignments get a zero gradient.                                                     */
int mms2ut_ctc_workspace_floats(int B, int T, int max_tgt_len, int64_t* n);
int mms2ut_ctc_loss_fwd(const mms2ut_half* logits, int64_t ld, int B, int T, int V, const int64_t* targets,
                        int64_t tgt_ld, int max_tgt_len, const int* in_len, const int* tgt_len, int blank,
                        int zero_infinity, float* work, float* loss_sum, hipStream_t stream);
int mms2ut_ctc_loss_bwd(const mms2ut_half* logits, int64_t ld, int B, int T, int V, const int64_t* targets,
                        int64_t tgt_ld, int max_tgt_len, const int* in_len, const int* tgt_len, int blank,
                        const float* work, const float* grad_scale, mms2ut_half* dlogits, int64_t ldd,
                        hipStream_t stream);
/* fairseq Trainer._check_grad_norms on device.  stage 0: buf[0..world) = 0 except
 * buf[rank] = ost[MMS_OST_GNORM]; the caller SUM-all-reduces buf; stage 1: ost[MMS_OST_INCONSISTENT]
 * = 1 when the norms are finite and max|n_r - n_0| / (n_0 + 1e-6) >= 1e-6 (sticky: never cleared)
 * — optim_prepare then sets MMS_OST_FATAL, which is sticky as well: from that step on no rank
 * updates anything (the host raises FloatingPointError on every rank at its next check).        */
int mms2ut_grad_norm_check(float* buf, int world, int rank, float* ost, int stage, hipStream_t stream);
/* x *= alpha in place (fp16, n % 8 == 0): the data-parallel gradient pre-division by world size
 * (torch DDP's allreduce hook divides each bucket before its SUM all-reduce)                    */
int mms2ut_scale_f16(mms2ut_half* x, int64_t n, float alpha, hipStream_t stream);
/* dst[0..n) = vals[0..n) (fp32, n <= 8; vals is a host array read at the call, passed to the
 * kernel as arguments): the trainer's per-step log vector (loss / nll / ntokens / nsentences /
 * sample size) initialised in one launch instead of a fill per slot                          */
int mms2ut_set_f32(float* dst, int n, const float* vals, hipStream_t stream);
/* acc (fp32) += x (fp16), n % 8 == 0: gradient accumulation over --update-freq micro-batches    */
int mms2ut_accum_f16_f32(float* acc, const mms2ut_half* x, int64_t n, hipStream_t stream);
int mms2ut_adam_fp16_master(mms2ut_half* param, const mms2ut_half* grad, float* master,
                            float* exp_avg, float* exp_avg_sq, int64_t n, const float* ost,
                            float beta1, float beta2, float eps, float weight_decay, hipStream_t stream);

/* ---------------------------------------------------------------- beam-search decoding
 * fairseq SequenceGenerator._generate (fairseq-generate --beam 10 --max-len-a 1, SURVEY §8f row 2;
 * scripts/textless/2_inference.sh:34-44).  log_softmax_step: log_softmax(logits.float()) of each
 * hypothesis row (get_normalized_probs) fused with the step's masking: NaN -> -inf, pad -> -inf,
 * mode 1 (step >= max_len): every token but eos -> -inf, mode 2 (step < min_len): eos -> -inf.
 * lprobs [rows][V] fp32.                                                                    */
int mms2ut_log_softmax_step(const mms2ut_half* logits, int64_t ld, int64_t rows, int V, int pad_idx,
                            int eos_idx, int mode, float* lprobs, hipStream_t stream);
/* One step of decoder self-attention against the K|V cache of one layer,
 * cache [slots][maxT][width = 2*H*hd] (K in columns [0, H*hd), V in [H*hd, 2*H*hd)), addressed
 * through slot [N][maxT] int32: key/value row t (t < T) of hypothesis n is row t of cache slot
 * slot[n][t] (beam reorders permute the table, not the cache).  T = *step + 1 is read on the
 * device (the step replays as a graph); row T-1 is this step's K|V, read from kv_new [N][ld_new]
 * and stored into row T-1 of slot n (slot[n][T-1] = n).  q [N][ldq] (head h at column h*hd),
 * out [N][ldo] fp16; softmax(scale q k^T) v per head in fp32.                                 */
int mms2ut_decode_self_attn(const mms2ut_half* q, int64_t ldq, mms2ut_half* cache, int32_t* slot, int N, int H,
                            int hd, int maxT, const int32_t* step, const mms2ut_half* kv_new, int64_t ld_new,
                            int64_t width, mms2ut_half* out, int64_t ldo, float scale, hipStream_t stream);
/* fairseq TransformerDecoder incremental embedding: x[n] = scale*E[tok[n]] + pos[pad+1+*step]
 * (E [V][D], pos sinusoid table [>= pad+2+step][D], fp16; step on the device).             */
int mms2ut_decode_embed(const int64_t* tok, const mms2ut_half* E, const mms2ut_half* pos, const int32_t* step,
                        int pad_idx, mms2ut_half* x, int N, int D, float scale, hipStream_t stream);
/* Decoder-step split-K epilogue: out[rows][cols] (fp16, row stride ldo) = act(sum of nsplit fp32
 * slabs [rows][cols] (slab elements apart) + bias) (+ aux, row stride ldaux); act = ReLU if relu.
 * bias / aux may be null.                                                                      */
int mms2ut_splitk_epilogue_f16(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                               const mms2ut_half* bias, const mms2ut_half* aux, int64_t ldaux, int relu,
                               mms2ut_half* out, int64_t ldo, hipStream_t stream);
/* The same reduction with the residual (aux required) followed by the next LayerNorm:
 * xout = fp16(fp16(sum of slabs + bias) + aux), y = LN(xout; gamma, beta, eps) — one launch,
 * bit-identical to mms2ut_splitk_epilogue_f16 + mms2ut_layernorm_fwd.  cols <= 1024.          */
int mms2ut_splitk_epilogue_ln_f16(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                                  const mms2ut_half* bias, const mms2ut_half* aux, int64_t ldaux,
                                  mms2ut_half* xout, int64_t ldx, const mms2ut_half* gamma,
                                  const mms2ut_half* beta, float eps, mms2ut_half* y, int64_t ldy,
                                  hipStream_t stream);
/* BeamSearch.step candidate selection: per sentence b, the top k (<= 32) of
 * lprobs[b*beam + j][v] + prev_scores[(b*beam + j) * ld_prev] over j < beam (j = 0 only when
 * first_step, prev_scores unused), v < V; descending, ties to the lower flat index j*V + v.
 * Outputs [bsz][k]: score (fp32), token v, beam j (int64).  work: bsz*32*k uint64 scratch
 * (two passes: 32 waves per sentence, then a merge).                                          */
int mms2ut_beam_topk(const float* lprobs, const float* prev_scores, int64_t ld_prev, int bsz, int beam, int V,
                     int first_step, int k, float* out_score, int64_t* out_tok, int64_t* out_beam,
                     uint64_t* work, hipStream_t stream);
/* reorder_incremental_state: src [L][Nsrc][maxT][width], dst [L][N][maxT][width] (each decoder
 * layer's self-attention K|V rows); dst[l][n][0:rows] = src[l][idx[n]][0:rows], idx[n] < Nsrc.
 * width % 8 == 0, 16-B aligned.                                                              */
int mms2ut_kv_cache_gather(const mms2ut_half* src, mms2ut_half* dst, const int64_t* idx, int L, int Nsrc,
                           int N, int maxT, int rows, int width, hipStream_t stream);

/* ---------------------------------------------------------------- fbank front end
 * fairseq get_fbank -> torchaudio.compliance.kaldi.fbank (audio_utils.py:326-349), 80 bins,
 * 25 ms / 10 ms, snip_edges, DC removal, pre-emphasis 0.97, povey window, 512-pt FFT, power,
 * mel (mel_banks: [nbins][257] fp32 dense table), log(max(x, FLT_EPS)); then utterance CMVN
 * (data-config feature transform) and zero-padded fp16 collation [B][Tmax][nbins]
 * (_collate_frames).  wave: concatenated fp32 samples (x 2^15), wave_off[B+1].              */
int mms2ut_fbank_frames(const int64_t* wave_off, int B, int32_t* n_frames_out, hipStream_t stream);
/* mel_range[2*m], mel_range[2*m+1]: first / one-past-last nonzero FFT bin of filter m; at most
 * 1024 nonzero weights over all filters (80 Kaldi bins: ~510)                                  */
int mms2ut_fbank_f32(const float* wave, const int64_t* wave_off, const int32_t* frame_off, int B,
                     int total_frames, const float* mel_banks, const int32_t* mel_range, int nbins,
                     float* feats, hipStream_t stream);
/* stats: caller-owned workspace of MMS_CMVN_WS_FLOATS(B, nbins) floats: [B][2][nbins] fp32
 * (per-utterance mean, std), then 8-B aligned fp64 slice partials [B][MMS_CMVN_SPLIT][2][nbins]   */
#define MMS_CMVN_SPLIT 8
#define MMS_CMVN_WS_FLOATS(B, nbins) ((((int64_t)2 * (B) * (nbins) + 1) & ~(int64_t)1) + \
                                      (int64_t)2 * (B) * MMS_CMVN_SPLIT * 2 * (nbins))
int mms2ut_fbank_cmvn_collate(const float* feats, const int32_t* frame_off, int B, int Tmax,
                              int nbins, int cmvn, float* stats, mms2ut_half* out, hipStream_t stream);
/* fairseq SpecAugmentTransform (feature_transforms/specaugment.py, the `specaugment` entry of
 * the data config's `_train` transforms, applied after utterance_cmvn by
 * speech_to_speech_dataset.py:271-272), in place on the collated features x [B][Tmax][nbins].
 * masks[b]: n_freq (f0, width) pairs then n_time (t0, width) pairs, drawn on the host; width 0 =
 * no mask.  use_const = 0: mask value = the utterance's mean over its valid [T][nbins] region
 * (the transform's mask_value=None default); otherwise mask_value.  Time warp is not built.   */
int mms2ut_specaugment_f16(mms2ut_half* x, const int32_t* frame_off, int B, int Tmax, int nbins,
                           const int32_t* masks, int n_freq, int n_time, int use_const,
                           float mask_value, hipStream_t stream);

/* ---------------------------------------------------------------- transformer layers
 * One whole pre-LN transformer layer per call — SURVEY §8b "encoder / decoder layer fwd/bwd":
 *   MMS_LAYER_ENC: fairseq TransformerEncoderLayer (encoder_normalize_before; A5, reached from
 *     S2TTransformerEncoder._forward at mm_s2s_transformer.py:464):
 *     x += drop(out_proj(MHA(LN1(x), key_len))); x += drop(fc2(drop(relu(fc1(LN3(x))))))
 *   MMS_LAYER_DEC: fairseq TransformerDecoderLayer (decoder_normalize_before; A10, reached at
 *     mm_s2s_transformer.py:693-696): causal self-attention block (LN1), cross-attention block
 *     (LN2, q_proj, K|V of the encoder output precomputed for all layers, out_proj), FFN (LN3).
 * The kernels are the ones the per-launch entries above run (GEMM epilogues, flash attention,
 * LayerNorm), enqueued in one call: forward on `s`; backward's dgrad chain on `main` and its
 * weight / bias / LayerNorm-parameter gradients on `side` (forked per job; side == main or NULL
 * runs them in order on main).  Dropout: rate and counter offset per site, one seed.
 * Buffers (the library never allocates): the forward writes what the backward needs and the
 * layer output into `saved` (mms2ut_layer_arena: byte offsets per MMS_SLOT_*); the backward writes
 * dx (and dropout(dx) when emit_p > 0) and every temporary into `scratch` (mms2ut_layer_scratch),
 * which the side stream reads — keep it (and `saved`) alive until the side stream is joined.
 * Split-K partials go to the per-stream workspaces sized by mms2ut_layer_ws.               */
enum { MMS_LAYER_ENC = 0, MMS_LAYER_DEC = 1 };
enum {
  MMS_SLOT_M1 = 0, MMS_SLOT_R1, MMS_SLOT_H1, MMS_SLOT_QKV, MMS_SLOT_LSE_SA, MMS_SLOT_O, MMS_SLOT_XA,
  MMS_SLOT_M2, MMS_SLOT_R2, MMS_SLOT_H2, MMS_SLOT_Q, MMS_SLOT_LSE_CA, MMS_SLOT_CO, MMS_SLOT_XB,
  MMS_SLOT_M3, MMS_SLOT_R3, MMS_SLOT_H3, MMS_SLOT_F1, MMS_SLOT_OUT, MMS_LAYER_NSLOT
};

typedef struct mms2ut_layer {
  int kind;                       /* MMS_LAYER_ENC / MMS_LAYER_DEC                               */
  int B, T, Tk, d, H, F;          /* T: the layer's length; Tk: cross-attention keys (decoder)   */
  float eps;
  const int32_t* self_len;        /* [B] self-attention key lengths                              */
  const int32_t* cross_len;       /* [B] decoder: encoder output lengths                         */
  /* parameters ([out, in] row-major fp16) */
  const mms2ut_half *ln1_g, *ln1_b, *w_qkv, *b_qkv, *w_o, *b_o;     /* self-attention block    */
  const mms2ut_half *ln2_g, *ln2_b, *w_cq, *b_cq, *w_co, *b_co;     /* cross-attention block   */
  const mms2ut_half* kv;          /* decoder: K | V of the encoder output [B*Tk] rows, ld_kv     */
  int64_t ld_kv;
  const mms2ut_half *ln3_g, *ln3_b, *w_fc1, *b_fc1, *w_fc2, *b_fc2; /* FFN block               */
  /* W^T images [in, out] of the dgrad weights, or NULL (transposed reads of W) */
  const mms2ut_half *wt_qkv, *wt_o, *wt_cq, *wt_co, *wt_fc1, *wt_fc2;
  /* gradients (views of the flat gradient buffer); g_ln*: [gamma | beta] */
  mms2ut_half *g_ln1, *g_w_qkv, *g_b_qkv, *g_w_o, *g_b_o;
  mms2ut_half *g_ln2, *g_w_cq, *g_b_cq, *g_w_co, *g_b_co;
  mms2ut_half *g_ln3, *g_w_fc1, *g_b_fc1, *g_w_fc2, *g_b_fc2;
  /* dropout: residual / attention-probability / activation rates, counter offsets per site */
  float p_drop, p_attn, p_act;
  uint64_t seed;
  uint64_t off_sa_attn, off_sa_res, off_ca_attn, off_ca_res, off_act, off_ffn_res;
  const mms2ut_half* x;           /* layer input [B*T, d]                                        */
  void* saved;                    /* forward arena; holds the output (MMS_SLOT_OUT)              */
} mms2ut_layer;

typedef struct mms2ut_layer_grad {
  const mms2ut_half* dy;          /* gradient of the layer output [B*T, d]                       */
  const mms2ut_half* dy_drop;     /* dropout(dy) with the FFN residual mask, or NULL             */
  float emit_p;                   /* > 0: also write dropout(dx) (the layer below's residual mask) */
  uint64_t emit_seed, emit_offset;
  mms2ut_half* dkv;               /* decoder: gradient of this layer's K | V columns, ld_dkv     */
  int64_t ld_dkv;
  void* scratch;
  float* main_ws;
  int64_t main_ws_floats;
  float* side_ws;
  int64_t side_ws_floats;
  int side_blocks;                /* grid cap of the grouped weight-gradient launch on the side   */
                                  /* stream (mms2ut_wgrad_group max_blocks; 0 = one per tile)      */
} mms2ut_layer_grad;

/* arena size (and the byte offset of every MMS_SLOT_*, -1 for slots the kind does not use)     */
int mms2ut_layer_arena(const mms2ut_layer* layer, int64_t* offsets, int64_t* bytes);
/* backward scratch size; dx_offsets[0] = dx, [1] = dropout(dx) (-1 unless emit_p > 0)          */
int mms2ut_layer_scratch(const mms2ut_layer* layer, float emit_p, int64_t* dx_offsets, int64_t* bytes);
/* floats of the main-stream (split-K fixup) and side-stream (weight-gradient slabs) workspaces   */
int mms2ut_layer_ws(const mms2ut_layer* layer, int64_t* main_floats, int64_t* side_floats);
int mms2ut_layer_fwd(const mms2ut_layer* layer, float* main_ws, int64_t main_ws_floats, hipStream_t stream);
int mms2ut_layer_bwd(const mms2ut_layer* layer, const mms2ut_layer_grad* grad, hipStream_t main,
                     hipStream_t side);
/* Launches the grouped weight gradients a layer backward held back (mms2ut_layer_bwd launches a
 * layer's group from inside the next layer's backward, behind its self-attention backward; env
 * MMS2UT_WGRAD_DEFER selects the point, 0 = no deferral), on the side stream behind `main`'s work
 * so far.  No-op when nothing is pending.  Call before joining the side stream or reporting a
 * gradient ready point (the host package does both).                                         */
int mms2ut_wgrad_flush(hipStream_t main);

/* ---------------------------------------------------------------- Conv1d subsampler
 * fairseq Conv1dSubsampler — SURVEY §8b mms2ut_conv1d_glu_{fwd,bwd} (A3; S2TTransformerEncoder's
 * front, reached at mm_s2s_transformer.py:464): nlayers x [Conv1d(C_l -> cout_l, k_l, stride 2,
 * padding k_l / 2) -> GLU over channels], input x [B][T][C] fp16 (row b*T + t), output
 * [B][T_out][cout_last / 2] at the arena offset conv1d_glu_arena returns.  One call enqueues the
 * layer sequence (im2col, projection GEMM with bias, GLU); the backward the GLU backward, the
 * weight / bias gradients on `side` (g_w[l] viewed [cout][C k], NULL = skip) and the input
 * gradients of layers > 0 (dgrad through wt[l] = W^T image [C k][cout] when non-NULL, col2im).
 * The first layer's input gradient is not formed (fbank features are not trained).  Buffers as for
 * the layers: arena (forward -> backward), scratch (keep until the side stream is joined),
 * per-stream workspaces from conv1d_glu_ws.                                                     */
#define MMS_CONV_MAX 4
typedef struct mms2ut_conv1d_glu {
  int B, T, C, nlayers;
  int k[MMS_CONV_MAX];            /* kernel sizes                                                */
  int cout[MMS_CONV_MAX];         /* conv output channels (2 x GLU channels), multiples of 16    */
  const mms2ut_half* w[MMS_CONV_MAX];    /* [cout][C_l][k] (nn.Conv1d weight)                   */
  const mms2ut_half* b[MMS_CONV_MAX];
  const mms2ut_half* wt[MMS_CONV_MAX];   /* W^T images [C_l k][cout] for the dgrads, or NULL     */
  mms2ut_half* g_w[MMS_CONV_MAX];
  mms2ut_half* g_b[MMS_CONV_MAX];
  const mms2ut_half* x;
  void* saved;
} mms2ut_conv1d_glu;
int mms2ut_conv1d_glu_arena(const mms2ut_conv1d_glu* c, int64_t* out_offset, int64_t* bytes);
/* dx_offset: the gradient of layer 1's input (= layer 0's GLU output) in the scratch, -1 for one layer */
int mms2ut_conv1d_glu_scratch(const mms2ut_conv1d_glu* c, int64_t* dx_offset, int64_t* bytes);
int mms2ut_conv1d_glu_ws(const mms2ut_conv1d_glu* c, int64_t* main_floats, int64_t* side_floats);
int mms2ut_conv1d_glu_fwd(const mms2ut_conv1d_glu* c, float* main_ws, int64_t main_ws_floats, hipStream_t stream);
int mms2ut_conv1d_glu_bwd(const mms2ut_conv1d_glu* c, const mms2ut_half* dy, void* scratch, float* main_ws,
                          int64_t main_ws_floats, float* side_ws, int64_t side_ws_floats, int side_blocks,
                          hipStream_t main, hipStream_t side);

/* ---------------------------------------------------------------- gated fusion
 * The fusion tail — SURVEY §8b mms2ut_gated_fusion_{fwd,bwd} (A6-A9: fuse_img_feat,
 * mm_s2s_transformer.py:594-622; SelectiveAttention fuse.py:65-117, MultimodalAttention =
 * nn.MultiheadAttention(add_bias_kv) fuse.py:145-167): image LayerNorm (image_pre_norm) +
 * SA_image dropout into a [B][Ti + extra][Di] key layout, SA_text dropout, q = text Wq^T + bq,
 * k|v = img Wkv^T + bkv (extra: + the bias_k|bias_v row per batch), one-head softmax attention
 * (key padding mask [B][>= Tk] uint8, 1 = padded; SA_attention dropout), out-projection, and either
 * the sigmoid gate (gate: merge = [attn_out | text], g = sigmoid(merge Wg^T + bg),
 * out = text + g (attn_out - text)) or the residual out = text + attn_out.  The output lives in
 * the arena (gated_fusion_arena's offset).  The backward writes d(text) (and with want_dimg the
 * image-feature gradient) into the scratch (offsets from gated_fusion_scratch) and the parameter
 * gradients (weight / bias gradients on `side`; g_ln / g_bias_kv are [gamma|beta], [k|v] spans).  */
typedef struct mms2ut_gated_fusion {
  int B, Te, Ti, Di, d;
  int extra;                      /* multimodal_attention (add_bias_kv); 0: selective_attention  */
  int gate;                       /* use_selective_gate                                          */
  int image_pre_norm;
  float eps;
  float p_img, p_txt, p_attn;     /* SA_image / SA_text / SA_attention dropout                  */
  uint64_t seed, off_img, off_txt, off_attn;
  const uint8_t* key_mask;        /* [B][ld_mask], 1 = padded image key, or NULL                 */
  int64_t ld_mask;
  const mms2ut_half *ln_g, *ln_b, *wq, *bq, *wkv, *bkv, *bias_kv, *wo, *bo, *wg, *bg;
  mms2ut_half *g_ln, *g_wq, *g_bq, *g_wkv, *g_bkv, *g_bias_kv, *g_wo, *g_bo, *g_wg, *g_bg;
  const mms2ut_half *wt_q, *wt_kv, *wt_o, *wt_g;   /* W^T images for the dgrads, or NULL        */
  const mms2ut_half* text;        /* [B*Te, d] encoder output                                    */
  const mms2ut_half* img;         /* [B*Ti, Di] image features                                   */
  void* saved;
} mms2ut_gated_fusion;
int mms2ut_gated_fusion_arena(const mms2ut_gated_fusion* f, int64_t* out_offset, int64_t* bytes);
/* offsets[0] = d(text), offsets[1] = d(img) (-1 without want_dimg)                             */
int mms2ut_gated_fusion_scratch(const mms2ut_gated_fusion* f, int want_dimg, int64_t* offsets, int64_t* bytes);
int mms2ut_gated_fusion_ws(const mms2ut_gated_fusion* f, int64_t* main_floats, int64_t* side_floats);
int mms2ut_gated_fusion_fwd(const mms2ut_gated_fusion* f, float* main_ws, int64_t main_ws_floats, hipStream_t stream);
int mms2ut_gated_fusion_bwd(const mms2ut_gated_fusion* f, const mms2ut_half* dres, int want_dimg, void* scratch,
                            float* main_ws, int64_t main_ws_floats, float* side_ws, int64_t side_ws_floats,
                            int side_blocks, hipStream_t main, hipStream_t side);

/* Buffer sizes of a coarse entry in one query: op MMS_OP_LAYER
 * (desc = mms2ut_layer*), MMS_OP_CONV1D_GLU (mms2ut_conv1d_glu*) or MMS_OP_GATED_FUSION
 * (mms2ut_gated_fusion*) -> sizes[0] forward arena bytes, [1] backward scratch bytes (layer: no
 * emitted dropout; fusion: without the image gradient), [2] main-stream and [3] side-stream
 * workspace floats.                                                                             */
enum { MMS_OP_LAYER = 0, MMS_OP_CONV1D_GLU = 1, MMS_OP_GATED_FUSION = 2 };
int mms2ut_workspace_size(int op, const void* desc, int64_t* sizes);

#ifdef __cplusplus
}
#endif
#endif /* MMS2UT_H */
