"""Micro-benchmark of the HIP GEMM on the training step's shapes (interleaved A/B of the two
paths in one process; random operands).  Usage: python scripts/gemm_bench.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels

M = 10000
SHAPES = [  # name, M, N, K, a_kc, b_kc, splitk
    ("qkv fwd", M, 2304, 768, True, True, 1),
    ("fc1 fwd", M, 3072, 768, True, True, 1),
    ("fc2 fwd", M, 768, 3072, True, True, 1),
    ("out fwd", M, 768, 768, True, True, 1),
    ("fc2 dgrad", M, 3072, 768, True, False, 1),
    ("fc1 dgrad", M, 768, 3072, True, False, 1),
    ("wgrad 3072x768", 3072, 768, M, False, False, 4),
    ("wgrad 3072x768 s8", 3072, 768, M, False, False, 8),
    ("wgrad 768x768", 768, 768, M, False, False, 15),
    ("wgrad 768x768 s8", 768, 768, M, False, False, 8),
    ("wgrad 768x768 s16", 768, 768, M, False, False, 16),
    ("conv2 fwd", 10000, 1536, 2560, True, True, 1),
    ("square 4096", 4096, 4096, 4096, True, True, 1),
    ("square 8192", 8192, 8192, 8192, True, True, 1),
]


def run(name, m, n, k, a_kc, b_kc, s, reps=20):
    A = torch.randn(m, k, device="cuda").half() if a_kc else torch.randn(k, m, device="cuda").half()
    B = torch.randn(n, k, device="cuda").half() if b_kc else torch.randn(k, n, device="cuda").half()
    if s > 1:
        C = torch.empty(s, m, n, dtype=torch.float32, device="cuda")
        epi = K.EPI_F32
    else:
        C = torch.empty(m, n, dtype=torch.float16, device="cuda")
        epi = K.EPI_F16
    res = {}
    for rnd in range(3):
        for path in ("reg", "dma", "dma2"):
            # reg: register-staged; dma: 3-stage LDS-DMA; dma2: 2-stage LDS-DMA (default)
            os.environ["MMS2UT_GEMM_PATH"] = path
            os.environ["MMS2UT_DMA_STAGES"] = "2"
            os.environ["MMS2UT_GEMM_BK"] = "32" if path == "dma" else "64"
            for _ in range(2):
                K.gemm(A, B, C, m, n, k, a_kc=a_kc, b_kc=b_kc, lda=A.stride(0), ldb=B.stride(0), ldc=n,
                       epi=epi, splitk=s, sCsplit=m * n)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                K.gemm(A, B, C, m, n, k, a_kc=a_kc, b_kc=b_kc, lda=A.stride(0), ldb=B.stride(0), ldc=n,
                       epi=epi, splitk=s, sCsplit=m * n)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / reps
            res[path] = min(res.get(path, 1e9), t)
    # hipBLASLt through torch on the same operands (C = A·B^T in our convention)
    At = A if a_kc else A.t()
    Bt = B.t() if b_kc else B
    for _ in range(3):
        torch.matmul(At, Bt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(At, Bt)
    e1.record()
    torch.cuda.synchronize()
    res["torch"] = e0.elapsed_time(e1) / reps
    fl = 2.0 * m * n * k
    print(f"{name:18s} M={m:6d} N={n:5d} K={k:6d}  torch {res['torch']*1e3:7.1f}us {fl/res['torch']/1e9:6.0f} TF"
          f"  reg {res['reg']*1e3:7.1f}us {fl/res['reg']/1e9:6.0f} TF"
          f"   bk32 {res['dma']*1e3:7.1f}us {fl/res['dma']/1e9:6.0f} TF"
          f"   dma2 {res['dma2']*1e3:7.1f}us {fl/res['dma2']/1e9:6.0f} TF", flush=True)
    os.environ.pop("MMS2UT_GEMM_PATH", None)


def epilogues(m=10000, n=768, k=768, reps=20):
    """Cost of the fused epilogues on the out-proj shape (register path)."""
    x = torch.randn(m, k, device="cuda").half()
    W = torch.randn(n, k, device="cuda").half()
    b = torch.randn(n, device="cuda").half()
    res = torch.randn(m, n, device="cuda").half()
    out = torch.empty(m, n, dtype=torch.float16, device="cuda")
    cases = [("plain", dict(epi=K.EPI_F16)), ("bias", dict(epi=K.EPI_F16, bias=b)),
             ("resid p=0", dict(epi=K.EPI_DROP_RESID, bias=b, aux=res)),
             ("resid p=.1", dict(epi=K.EPI_DROP_RESID, bias=b, aux=res, p=0.1, drop=(1, 0))),
             ("relu p=.1", dict(epi=K.EPI_RELU_DROP, bias=b, p=0.1, drop=(1, 0)))]
    for name, kw in cases:
        for _ in range(2):
            K.linear(x, W, out=out, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            K.linear(x, W, out=out, **kw)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps
        print(f"epilogue {name:12s} {t*1e3:7.1f}us {2.0*m*n*k/t/1e9:6.0f} TF", flush=True)


if __name__ == "__main__":
    for sh in SHAPES:
        run(*sh)
    epilogues()
    epilogues(n=3072)
