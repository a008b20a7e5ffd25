// Short-M NT GEMM (decoder tokens, M ~ 200-2000 rows) with the fused epilogues — included by
// gemm.hip inside its anonymous namespace.
//
// At M ~ 470 a 128x128-tile grid covers a few dozen CUs, and the time of every route is set by
// memory latency, not by MFMA: a 128x128 block walking K = 768 in 12 pipelined k-steps takes ~10 us,
// the split-K slabs + fixup route pays two launches.  This kernel issues ALL of a block's operand
// loads at once — global -> VGPR in the MFMA fragment layout (lane l: row l&15, 8 k from 8*(l>>4)),
// no LDS staging, no k-loop — so a block costs one load latency plus its bytes:
//   * block tile 16*TM x 16*TN (64x64, 32x64 or 32x32), K split S ways across blocks;
//   * the block's four waves take interleaved 64-wide k-chunks of the split (wave w: w, w+4, ...,
//     NLOC chunks each), each accumulating the whole tile; the four partial tiles are summed through
//     LDS in wave order;
//   * S == 1: the epilogue runs right there;  S > 1: the block writes its fp32 partial tile to the
//     workspace, and the LAST of the tile's S blocks to arrive (one atomic ticket per tile; all S
//     blocks of a tile run on one XCD, so the partials meet in its L2) sums the S partials in split
//     order and runs the epilogue, then re-arms the ticket (0) for the next launch on the stream.
//     Split order and wave order are fixed, so results do not depend on scheduling.
// Rows past M / columns past N read a clamped (valid) row and are dropped at the store.
// Requires A and B K-contiguous, K % (256 * NLOC * S) == 0, batch 1 (host routing: skinny_pick).

template <int EPI, int TM, int TN, int NLOC>
__global__ void __launch_bounds__(NT, 2) gemm_skinny_kernel(GemmP P, int tiles_m, int tiles_n, int nsplit,
                                                             float* __restrict__ part, int* __restrict__ ticket) {
  constexpr int BMS = 16 * TM, BNS = 16 * TN, LDR = BNS + 4;   // LDR: padded fp32 row of the reduction tile
  __shared__ __attribute__((aligned(16))) float red[4 * BMS * LDR];
  __shared__ int is_last;
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  // XCD-aware order (workgroups go round-robin over the 8 XCDs, bid % 8): XCD x owns one contiguous
  // range of column-major tiles (tiles sharing a weight slice share its L2) with ALL splits of each
  // of them, so a tile's partials meet in one L2 — no cross-XCD traffic, no L2 writeback/invalidate.
  // The grid is 8 x (longest range) x nsplit; blocks past a shorter range only stamp.
  const int T = tiles_m * tiles_n, q = T / 8, r = T % 8;
  const int x = blockIdx.x % 8, j = blockIdx.x / 8;
  const int lt = j / nsplit, split = j % nsplit;
  if (lt >= q + (x < r ? 1 : 0)) {
    stamp_end(P.stamps, t_start);
    return;
  }
  const int tile = x * q + min(x, r) + lt;
  const int tm = tile % tiles_m, tn = tile / tiles_m;
  const int bm = tm * BMS, bn = tn * BNS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k0 = split * (NLOC * 256) + 64 * w + 8 * (lane >> 4);

  s16x8 ra[NLOC][TM][2], rb[NLOC][TN][2];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const h16* pa = P.A + (long)min(bm + 16 * i + (lane & 15), P.M - 1) * P.lda + k0;
#pragma unroll
    for (int c = 0; c < NLOC; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) ra[c][i][h] = *reinterpret_cast<const s16x8*>(pa + 256 * c + 32 * h);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const h16* pb = P.B + (long)min(bn + 16 * j + (lane & 15), P.N - 1) * P.ldb + k0;
#pragma unroll
    for (int c = 0; c < NLOC; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) rb[c][j][h] = *reinterpret_cast<const s16x8*>(pb + 256 * c + 32 * h);
  }

  // every load is in flight before the first MFMA waits (the scheduler would otherwise interleave
  // loads with MFMAs to save registers and serialise the latencies)
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NLOC; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h16x8, rb[c][j][h]),
                                                             __builtin_bit_cast(h16x8, ra[c][i][h]), acc[i][j], 0, 0, 0);

  // (B, A) operand order: lane l holds C(16i + (l&15), 16j + 4(l>>4) + e), e = 0..3
  float* mine = red + w * BMS * LDR;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      *reinterpret_cast<f32x4*>(mine + (16 * i + (lane & 15)) * LDR + 16 * j + 4 * (lane >> 4)) = acc[i][j];
  __syncthreads();

  // the block's tile summed over its four waves (wave order), 8 consecutive columns per item
  auto wave_sum = [&](int row, int c8, float (&v)[8]) {
    const float* src = red + row * LDR + c8;
    const f32x4 lo0 = *reinterpret_cast<const f32x4*>(src), hi0 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = lo0[e]; v[e + 4] = hi0[e]; }
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src + ww * BMS * LDR);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + ww * BMS * LDR + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] += lo[e]; v[e + 4] += hi[e]; }
    }
  };
  constexpr int ITEMS = BMS * BNS / 8;
  if (nsplit == 1) {
    for (int o = threadIdx.x; o < ITEMS; o += NT) {
      const int row = o / (BNS / 8), c8 = (o % (BNS / 8)) * 8;
      float v[8];
      wave_sum(row, c8, v);
      epilogue_store8<EPI>(P, P.C, P.aux, bm + row, bn + c8, v);
    }
    stamp_end(P.stamps, t_start);
    return;
  }

  // split-K: partial tile -> workspace [tile][split][BMS x BNS]; the last arrival reduces
  float* tile_part = part + (long)tile * nsplit * (BMS * BNS);
  for (int o = threadIdx.x; o < ITEMS; o += NT) {
    const int row = o / (BNS / 8), c8 = (o % (BNS / 8)) * 8;
    float v[8];
    wave_sum(row, c8, v);
    float* dst = tile_part + (long)split * (BMS * BNS) + row * BNS + c8;
    *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
  // Release: every thread's partial stores have completed (acknowledged by the XCD's L2, the one
  // all the tile's splits share) before the ticket is taken.  No agent-scope fence: on this chip it
  // writes back / invalidates the whole L2 (measured: 60-100 us per block).  The reducing block reads
  // the partials from that L2 — its L1 never held those lines in this launch (invalidated at kernel
  // start, never read since).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) is_last = atomicAdd(ticket + tile, 1) == nsplit - 1;
  __syncthreads();
  if (is_last) {
    for (int o = threadIdx.x; o < ITEMS; o += NT) {
      const int row = o / (BNS / 8), c8 = (o % (BNS / 8)) * 8;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const float* src = tile_part + row * BNS + c8;
      // four splits' loads in flight at a time (indices clamped: the loads are unconditional, the
      // adds of clamped duplicates are skipped), summed in split order
      for (int s0 = 0; s0 < nsplit; s0 += 4) {
        f32x4 lo[4], hi[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long off = (long)min(s0 + u, nsplit - 1) * (BMS * BNS);
          lo[u] = *reinterpret_cast<const f32x4*>(src + off);
          hi[u] = *reinterpret_cast<const f32x4*>(src + off + 4);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (s0 + u < nsplit)
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[e] += lo[u][e]; v[e + 4] += hi[u][e]; }
      }
      epilogue_store8<EPI>(P, P.C, P.aux, bm + row, bn + c8, v);
    }
    if (threadIdx.x == 0) ticket[tile] = 0;   // re-armed for the next launch (stream-ordered)
  }
  stamp_end(P.stamps, t_start);
}
