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
//     workspace and the LAST of the tile's S blocks to arrive (one atomic ticket per tile) sums the
//     S partials in split order and runs the epilogue, then re-arms the ticket (0) for the next
//     launch on the stream.  Split order and wave order are fixed, so results do not depend on
//     scheduling or placement.
// The partial-tile hand-off is placement-independent (cdna_hip_programming.md §6 Guideline 16, the
// split-K recipe's write-through form): partials are stored sc1 (write-through, no release fence
// needed), every storing wave drains (vmcnt(0)) before the block's barrier, one lane takes the
// ticket (relaxed agent-scope atomic), and the reducer reads EVERY partial with sc1 loads (L1
// bypassed, so no stale line of this CU can be read).  Keeping a tile's splits on one XCD (the
// bid % 8 ranges below) is a speed choice only; `scatter` deals them over different XCDs (tests).
// Rows past M / columns past N read a clamped (valid) row and are dropped at the store.
// Requires A and B K-contiguous, K % (256 * NLOC * S) == 0, batch 1 (host routing: skinny_pick).

typedef unsigned int sk_u32x4 __attribute__((ext_vector_type(4)));

template <int EPI, int TM, int TN, int NLOC>
__global__ void __launch_bounds__(NT, 2) gemm_skinny_kernel(GemmP P, int tiles_m, int tiles_n, int nsplit,
                                                             float* __restrict__ part, int* __restrict__ ticket,
                                                             int scatter, int* __restrict__ xcc_out) {
  constexpr int BMS = 16 * TM, BNS = 16 * TN, LDR = BNS + 4;   // LDR: padded fp32 row of the reduction tile
  __shared__ __attribute__((aligned(16))) float red[4 * BMS * LDR];
  __shared__ int is_last;
  const unsigned long long t_start = P.stamps ? stamp_now() : 0ull;
  if (P.thresh) P.seed = mms_step_seed(P.seed);
  // XCD-aware order (workgroups are observed to go round-robin over the 8 XCDs, bid % 8): group x
  // owns one contiguous range of column-major tiles (tiles sharing a weight slice share an L2) with
  // ALL splits of each of them, so a tile's partials stay in one L2 — a speed choice, the hand-off
  // below is correct for any placement.  scatter != 0 puts split s of a tile in group (owner + s) % 8
  // instead (tests: the splits then meet across XCDs).  The grid is 8 x (longest range) x nsplit;
  // blocks past a shorter range only stamp.
  const int T = tiles_m * tiles_n, q = T / 8, r = T % 8;
  const int x = blockIdx.x % 8, j = blockIdx.x / 8;
  const int lt = j / nsplit, split = j % nsplit;
  const int owner = scatter ? (x + 8 * nsplit - split) % 8 : x;
  if (xcc_out && threadIdx.x == 0) xcc_out[blockIdx.x] = (int)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));
  if (lt >= q + (owner < r ? 1 : 0)) {
    stamp_end(P.stamps, t_start);
    return;
  }
  const int tile = owner * q + min(owner, r) + lt;
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

  // split-K: partial tile -> workspace [tile][split][BMS x BNS], written through (sc1)
  float* tile_part = part + (long)tile * nsplit * (BMS * BNS);
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      (void*)tile_part, (short)0, (int)((long)nsplit * BMS * BNS * 4), 0x00020000);
  for (int o = threadIdx.x; o < ITEMS; o += NT) {
    const int row = o / (BNS / 8), c8 = (o % (BNS / 8)) * 8;
    float v[8];
    wave_sum(row, c8, v);
    const int off = ((split * (BMS * BNS)) + row * BNS + c8) * 4;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sk_u32x4, f32x4{v[0], v[1], v[2], v[3]}), rp, off, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sk_u32x4, f32x4{v[4], v[5], v[6], v[7]}), rp, off + 16, 0, 16);
  }
  // every storing wave drains its write-through stores, then ONE lane takes the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    is_last = __hip_atomic_fetch_add(ticket + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
  __syncthreads();
  if (is_last) {
    for (int o = threadIdx.x; o < ITEMS; o += NT) {
      const int row = o / (BNS / 8), c8 = (o % (BNS / 8)) * 8;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int src = (row * BNS + c8) * 4;
      // four splits' loads in flight at a time (indices clamped: the loads are unconditional, the
      // adds of clamped duplicates are skipped), summed in split order; every load sc1
      for (int s0 = 0; s0 < nsplit; s0 += 4) {
        f32x4 lo[4], hi[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int off = src + min(s0 + u, nsplit - 1) * (BMS * BNS * 4);
          lo[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, 16));
          hi[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, off + 16, 0, 16));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (s0 + u < nsplit)
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[e] += lo[u][e]; v[e + 4] += hi[u][e]; }
      }
      epilogue_store8<EPI>(P, P.C, P.aux, bm + row, bn + c8, v);
    }
    // re-armed for the next launch on the stream (every block of this tile has taken its ticket)
    if (threadIdx.x == 0) __hip_atomic_store(ticket + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  stamp_end(P.stamps, t_start);
}
