"""Isolated A/B of the 128x128 NT kernel (tall mode 0) against the 160 x 128 one (mode 2) and the
192 x 128 one (mode 3) and the shape rule (mode 1) on the step's M x N x K shapes around the 512-slot round boundary; random fp16,
warm, HIP events over 20 launches.  usage: python scripts/gemm_tall_ab.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for M in (4000, 6000, 7000, 10000, 12000):
    for N, Kd, name in ((768, 768, "DROP_RESID"), (768, 2304, "F16"), (768, 3072, "F16"), (768, 3072, "DROP_RESID"),
                        (2304, 768, "F16"), (3072, 768, "RELU_DROP")):
        g = torch.Generator(device="cuda").manual_seed(M + N + Kd)
        x = (torch.randn(M, Kd, device="cuda", generator=g) * 0.5).half()
        W = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).half()
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
        aux = torch.randn(M, N, device="cuda", generator=g).half()
        out = torch.empty(M, N, dtype=torch.float16, device="cuda")
        epi = getattr(K, "EPI_" + name)
        res = {}
        for mode in (0, 2, 3, 5, 1):
            K.call("mms2ut_gemm_set_tall", mode)
            res[mode] = timeit(lambda: K.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, epi=epi, bias=b,
                                              aux=aux if name == "DROP_RESID" else None, ldaux=N,
                                              p=0.1 if name != "F16" else 0.0, seed=3, offset=0, ld_rng=N,
                                              fixup=False))
        K.call("mms2ut_gemm_set_tall", 1)
        tf = 2.0 * M * N * Kd / 1e12
        print(f"M={M:5d} N={N:4d} K={Kd:4d} {name:11s} t128 {res[0]:6.1f} us ({tf / res[0] * 1e6:5.0f} TF)  "
              f"t160 {res[2]:6.1f} us ({tf / res[2] * 1e6:5.0f} TF)  t192 {res[3]:6.1f}  t96 {res[5]:6.1f}  rule {res[1]:6.1f}",
              flush=True)
