"""GPU: the bench's live GEMM timing.  In stamp mode every GEMM kernel's workgroups record start /
end s_memrealtime ticks; a launch's duration (max end - min start) must be positive, bounded by
the HIP-event time around the same launches, and the recorded block ranges must tile the buffer
(a split-K fixup's blocks follow its GEMM's)."""
import importlib

import numpy as np
import pytest
import torch

mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels

pytestmark = pytest.mark.gpu


def test_stamp_durations_bounded_by_events():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    shapes = [(4096, 3072, 768), (2000, 768, 768), (470, 768, 3072)]   # last one takes the split-K fixup path
    xs = [(torch.randn(m, k, device=dev).half(), (0.05 * torch.randn(n, k, device=dev)).half()) for m, n, k in shapes]
    outs = [torch.empty(m, n, device=dev, dtype=torch.float16) for m, n, k in shapes]
    for (x, W), o in zip(xs, outs):      # warm the kernels (first-launch code load)
        K.linear(x, W, out=o)
    torch.cuda.synchronize()
    stamps = torch.zeros(2 * 100_000, dtype=torch.int64, device=dev)
    K.gemm_profile_begin(100)
    K.gemm_profile_stamps(stamps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for (x, W), o in zip(xs, outs):
        K.linear(x, W, out=o)
    e1.record()
    torch.cuda.synchronize()
    _, n, _, _ = K.gemm_profile_end()
    assert n == len(shapes)
    d = K.gemm_profile_durations(stamps, n)
    assert np.isfinite(d).all() and (d > 0).all(), d
    assert d.sum() <= e0.elapsed_time(e1) * 1.02 + 0.005, (d, e0.elapsed_time(e1))
    # the same outputs as an unprofiled run (instrumentation does not touch results)
    for (x, W), o in zip(xs, outs):
        ref = torch.empty_like(o)
        K.linear(x, W, out=ref)
        assert torch.equal(ref, o)


def test_stamp_overflow_reported():
    dev = torch.device("cuda")
    x = torch.randn(4096, 768, device=dev).half()
    W = (0.05 * torch.randn(3072, 768, device=dev)).half()
    o = torch.empty(4096, 3072, device=dev, dtype=torch.float16)
    stamps = torch.zeros(2 * 8, dtype=torch.int64, device=dev)    # room for 8 workgroups only
    K.gemm_profile_begin(10)
    K.gemm_profile_stamps(stamps)
    K.linear(x, W, out=o)
    torch.cuda.synchronize()
    _, n, _, _ = K.gemm_profile_end()
    d = K.gemm_profile_durations(stamps, n)
    assert n == 1 and np.isnan(d[0])
