"""Isolated cost of each fused GEMM epilogue on the step's large shapes (128x128 path).
usage: python scripts/epi_bench.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


M, d, F = 8704, 768, 3072
x = torch.randn(M, d, device="cuda").half()
W1 = (0.05 * torch.randn(F, d, device="cuda")).half()
b1 = torch.randn(F, device="cuda").half()
f1 = torch.randn(M, F, device="cuda").half()
dy = torch.randn(M, d, device="cuda").half()
W2 = (0.05 * torch.randn(d, F, device="cuda")).half()
out = torch.empty(M, F, dtype=torch.float16, device="cuda")
fl = 2.0 * M * F * d
cases = [
    ("fc1 fwd plain", lambda: K.linear(x, W1, out=out)),
    ("fc1 fwd bias", lambda: K.linear(x, W1, b1, out=out)),
    ("fc1 fwd relu p=0", lambda: K.linear(x, W1, b1, out=out, epi=K.EPI_RELU_DROP)),
    ("fc1 fwd relu-drop p=.1", lambda: K.linear(x, W1, b1, out=out, epi=K.EPI_RELU_DROP, p=0.1, drop=(1, 0))),
    ("fc2 dgrad plain", lambda: K.linear_dgrad(dy, W2, out=out)),
    ("fc2 dgrad relu-bwd", lambda: K.linear_dgrad(dy, W2, out=out, epi=K.EPI_RELU_DROP_BWD, aux=f1, p=0.1)),
]
for name, fn in cases:
    us = t(fn)
    print(f"{name:24s} {us:7.1f} us  {fl / us / 1e6:6.0f} TF", flush=True)
