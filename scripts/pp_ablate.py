"""Isolated timings of the ping-pong GEMM at forced tile heights on three step shapes (for the
ablation builds of gemm_pp.hip: -DMMS_PP_NODMA / NOREAD / NOMFMA, loaded through MMS2UT_LIB).
usage: MMS2UT_LIB=... python scripts/pp_ablate.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
line = []
for M, N, Kd, bm in ((10000, 3072, 768, 256), (10000, 768, 3072, 128), (12000, 768, 3072, 192), (8192, 8192, 8192, 256)):
    x = (torch.randn(M, Kd, device="cuda") * 0.5).half()
    W = (torch.randn(N, Kd, device="cuda") * 0.05).half()
    out = torch.empty(M, N, dtype=torch.float16, device="cuda")
    K.call("mms2ut_gemm_set_pp", bm)
    run = lambda: K.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, fixup=False)  # noqa: E731
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    line.append(f"{M}x{N}x{Kd}/pp{bm} {us:7.1f} us ({2.0 * M * N * Kd / us / 1e6:5.0f} TF)")
K.call("mms2ut_gemm_set_pp", -1)
print("  ".join(line), flush=True)
