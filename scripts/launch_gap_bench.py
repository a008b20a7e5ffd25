"""Dependent back-to-back kernel cost on one stream: N small kernels (a) launched eagerly,
(b) captured once into a HIP graph and replayed; plus a GEMM-sized chain.  Shows how much of the
step's ~6 us per-kernel gap a graph removes."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels


def chain(x, y, n):
    for _ in range(n):
        K.call("mms2ut_add_f16", x.data_ptr(), y.data_ptr(), y.data_ptr(), x.numel(), K._s())


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


# GPU-side gap with the host far ahead: a long GEMM first, then the chain queued behind it
A = torch.randn(8192, 8192, device="cuda").half()
C = torch.empty_like(A)
for numel in (1 << 12, 1 << 20):
    x = torch.randn(numel, device="cuda").half()
    y = torch.zeros_like(x)
    n = 200
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        K.gemm(A, A, C, 8192, 8192, 8192, lda=8192, ldb=8192, ldc=8192)
    e0.record()
    chain(x, y, n)
    e1.record()
    torch.cuda.synchronize()
    print(f"host-ahead numel {numel:9d}: {e0.elapsed_time(e1) * 1e3 / n:6.2f} us/kernel", flush=True)

for numel in (1 << 12, 1 << 20, 1 << 24):
    x = torch.randn(numel, device="cuda").half()
    y = torch.zeros_like(x)
    n = 200
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eager = timed(lambda: chain(x, y, n))
        g = torch.cuda.CUDAGraph()
        chain(x, y, 2)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            chain(x, y, n)
        graph = timed(lambda: g.replay())
    print(f"numel {numel:9d}: eager {eager / n:6.2f} us/kernel   graph {graph / n:6.2f} us/kernel", flush=True)
