#include <stdlib.h>
// Error plumbing + split-K reduction.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"
#include "../../include/mms2ut.h"

namespace mms {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}
}  // namespace mms

extern "C" const char* mms2ut_last_error(void) { return mms::g_err; }
extern "C" int mms2ut_version(void) { return 1; }

// A non-blocking stream at a clamped priority (lower = more urgent).  The step's own streams are
// created here so that no work on the legacy default stream implicitly waits for them (a stream
// created without hipStreamNonBlocking synchronises with the NULL stream in both directions).
extern "C" int mms2ut_stream_create(int priority, hipStream_t* out) {
  if (!out) {
    mms::set_error("stream_create: null out");
    return 1;
  }
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
  const int p = priority < greatest ? greatest : (priority > least ? least : priority);
  const hipError_t e = hipStreamCreateWithPriority(out, hipStreamNonBlocking, p);
  if (e != hipSuccess) {
    mms::set_error("stream_create: %s", hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" int mms2ut_stream_destroy(hipStream_t stream) {
  if (!stream) {
    mms::set_error("stream_destroy: null stream");
    return 1;
  }
  const hipError_t e = hipStreamDestroy(stream);
  if (e != hipSuccess) {
    mms::set_error("stream_destroy: %s", hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

namespace {
__global__ void splitk_reduce_kernel(const float* __restrict__ slabs, int nsplit, long slab,
                                     int rows, int cols, void* out, long ldo, int out_f16,
                                     float alpha, const float* __restrict__ rs_slabs, h16* __restrict__ rs_out) {
  const long n4 = (long)rows * (cols / 4);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long r = i / (cols / 4), c = (i % (cols / 4)) * 4;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nsplit; ++k)
      s += *reinterpret_cast<const f32x4*>(slabs + k * slab + r * cols + c);
    s *= alpha;
    // mode bit0: fp16 output (else fp32); bit1: accumulate into the output
    if (out_f16 & 1) {
      h16x4* o = reinterpret_cast<h16x4*>(reinterpret_cast<h16*>(out) + r * ldo + c);
      if (out_f16 & 2) { h16x4 p = *o; s += f32x4{(float)p[0], (float)p[1], (float)p[2], (float)p[3]}; }
      *o = h16x4{(h16)s[0], (h16)s[1], (h16)s[2], (h16)s[3]};
    } else {
      f32x4* o = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + r * ldo + c);
      if (out_f16 & 2) s += *o;
      *o = s;
    }
  }
  // optional tail: the bias-gradient partials [nsplit][rows] -> rs_out fp16 (overwrite)
  if (rs_slabs) {
    const long m4 = rows / 4;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < m4; i += (long)gridDim.x * blockDim.x) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < nsplit; ++k) s += *reinterpret_cast<const f32x4*>(rs_slabs + (long)k * rows + 4 * i);
      s *= alpha;
      *reinterpret_cast<h16x4*>(rs_out + 4 * i) = h16x4{(h16)s[0], (h16)s[1], (h16)s[2], (h16)s[3]};
    }
  }
}
}  // namespace

extern "C" int mms2ut_splitk_reduce(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                                    void* out, int64_t ldo, int out_f16, float alpha,
                                    hipStream_t stream) {
  MMS_REQUIRE(cols % 4 == 0 && ldo % 4 == 0, "splitk_reduce: cols/ldo must be multiples of 4");
  const long n4 = (long)rows * (cols / 4);
  if (n4 == 0) return 0;
  int grid = (int)((n4 + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, stream, slabs, nsplit, slab,
                     rows, cols, out, ldo, out_f16, alpha, (const float*)nullptr, (h16*)nullptr);
  return mms::check_launch("splitk_reduce");
}

extern "C" int mms2ut_splitk_reduce_bias(const float* slabs, int nsplit, int64_t slab, int rows, int cols,
                                         mms2ut_half* out, int64_t ldo, const float* rs_slabs,
                                         mms2ut_half* rs_out, hipStream_t stream) {
  MMS_REQUIRE(cols % 4 == 0 && ldo % 4 == 0 && rows % 4 == 0,
              "splitk_reduce_bias: rows/cols/ldo must be multiples of 4");
  MMS_REQUIRE(rs_slabs && rs_out && ((uintptr_t)rs_out & 7) == 0, "splitk_reduce_bias: bad bias buffers");
  const long n4 = (long)rows * (cols / 4);
  if (n4 == 0) return 0;
  int grid = (int)((n4 + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, stream, slabs, nsplit, slab,
                     rows, cols, (void*)out, ldo, 1, 1.f, rs_slabs, rs_out);
  return mms::check_launch("splitk_reduce_bias");
}

// ------------------------------------------------------------------------------------------
// stream fork/join for the weight-gradient side stream: `waiter` waits for everything enqueued
// on `signaler` so far.  A small ring of timing-disabled events (created once per process) is
// re-recorded round-robin; a wait binds to the record that precedes it, so reuse is safe.
// The events skip the system-scope fence (hipEventDisableSystemFence): both streams are on this
// device, whose kernels already release / acquire at device scope, and the default system-scope
// release made every fork a full cache writeback — a ~7 us bubble on the main stream after each
// layer's LayerNorm backward, ~1 ms per step (round-5 trace, profiles/round5_fork_fence.txt).
// ------------------------------------------------------------------------------------------
namespace {
constexpr int kEvRing = 64;
hipEvent_t g_ev[kEvRing];
int g_ev_n = -1, g_ev_i = 0;
}  // namespace

extern "C" int mms2ut_stream_wait(hipStream_t waiter, hipStream_t signaler) {
  if (waiter == signaler) return 0;
  if (g_ev_n < 0) {
    const char* e = getenv("MMS2UT_FORK_SYSTEM_FENCE");   // 1: the default system-scope events (A/B)
    const unsigned flags = hipEventDisableTiming | (e && atoi(e) ? 0u : (unsigned)hipEventDisableSystemFence);
    for (int i = 0; i < kEvRing; ++i)
      if (hipEventCreateWithFlags(&g_ev[i], flags) != hipSuccess) {
        mms::set_error("stream_wait: hipEventCreate failed");
        return 1;
      }
    g_ev_n = kEvRing;
  }
  hipEvent_t e = g_ev[g_ev_i];
  g_ev_i = (g_ev_i + 1) % kEvRing;
  if (hipEventRecord(e, signaler) != hipSuccess || hipStreamWaitEvent(waiter, e, 0) != hipSuccess) {
    mms::set_error("stream_wait: record/wait failed");
    return 1;
  }
  return 0;
}

// Device-scope events for ordering this process's streams on one GPU (same flags as the fork ring):
// deferred optimizer chunks -> the next forward, weight-transpose refresh -> dgrad, per-group
// gradient hand-offs.  No timing, no host synchronisation.
extern "C" int mms2ut_event_create(hipEvent_t* out) {
  MMS_REQUIRE(out != nullptr, "event_create: null out");
  const char* e = getenv("MMS2UT_FORK_SYSTEM_FENCE");
  const unsigned flags = hipEventDisableTiming | (e && atoi(e) ? 0u : (unsigned)hipEventDisableSystemFence);
  const hipError_t r = hipEventCreateWithFlags(out, flags);
  MMS_REQUIRE(r == hipSuccess, "event_create: %s", hipGetErrorString(r));
  return 0;
}
extern "C" int mms2ut_event_record(hipEvent_t ev, hipStream_t stream) {
  const hipError_t r = hipEventRecord(ev, stream);
  MMS_REQUIRE(r == hipSuccess, "event_record: %s", hipGetErrorString(r));
  return 0;
}
extern "C" int mms2ut_event_wait(hipStream_t stream, hipEvent_t ev) {
  const hipError_t r = hipStreamWaitEvent(stream, ev, 0);
  MMS_REQUIRE(r == hipSuccess, "event_wait: %s", hipGetErrorString(r));
  return 0;
}
extern "C" int mms2ut_event_destroy(hipEvent_t ev) {
  const hipError_t r = hipEventDestroy(ev);
  MMS_REQUIRE(r == hipSuccess, "event_destroy: %s", hipGetErrorString(r));
  return 0;
}

// ------------------------------------------------------------------------------------------
// Step-seed indirection (HIP-graph replay of the training step; common.h mms_step_seed).
// ------------------------------------------------------------------------------------------
namespace mms {
int bind_step_seed_gemm(const uint64_t* d);
int bind_step_seed_attention(const uint64_t* d);
int bind_step_seed_ops(const uint64_t* d);
}  // namespace mms

extern "C" int mms2ut_bind_step_seed(const uint64_t* delta) {
  if (mms::bind_step_seed_gemm(delta) || mms::bind_step_seed_attention(delta) || mms::bind_step_seed_ops(delta) ||
      mms_bind_step_seed_tu(delta)) {
    mms::set_error("bind_step_seed: hipMemcpyToSymbol failed");
    return 1;
  }
  return 0;
}

namespace {
__global__ void step_seed_advance_kernel(uint64_t* delta, uint64_t inc) {
  if (threadIdx.x == 0) delta[0] += inc;
}
}  // namespace

extern "C" int mms2ut_step_seed_advance(uint64_t* delta, uint64_t inc, hipStream_t s) {
  MMS_REQUIRE(delta, "step_seed_advance: null delta");
  hipLaunchKernelGGL(step_seed_advance_kernel, dim3(1), dim3(64), 0, s, delta, inc);
  return mms::check_launch("step_seed_advance");
}

