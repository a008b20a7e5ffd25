"""Segment timing of the ping-pong GEMM (diagnostic build: scripts/build_ab.sh ppdiag gemm_pp.hip
-DMMS_PP_DIAG, loaded through MMS2UT_LIB): per row group, mean s_memtime cycles per 32-deep slot in
each loop segment, averaged over blocks, plus the isolated kernel time.
usage: MMS2UT_LIB=... python scripts/pp_diag.py"""
import ctypes as C
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels
lib = mm._lib.load() if hasattr(mm._lib, "load") else None
cdll = C.CDLL(mm._lib.LIB_PATH)
buf = torch.zeros(4096 * 2 * 8, dtype=torch.int64, device="cuda")
assert cdll.mms2ut_pp_diag_bind(C.c_void_p(buf.data_ptr())) == 0
for M, N, Kd, bm in ((10000, 768, 3072, 128), (10000, 3072, 768, 256), (10000, 2304, 768, 192), (12000, 768, 3072, 192)):
    x = (torch.randn(M, Kd, device="cuda") * 0.5).half()
    W = (torch.randn(N, Kd, device="cuda") * 0.05).half()
    out = torch.empty(M, N, dtype=torch.float16, device="cuda")
    K.call("mms2ut_gemm_set_pp", bm)
    for _ in range(3):
        K.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, fixup=False)
    buf.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    K.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, fixup=False)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3
    tiles = -(-M // bm) * -(-N // 256)
    d = buf.view(-1, 2, 8)[:tiles].cpu().numpy().astype(np.float64)
    print(f"M={M} N={N} K={Kd} BM={bm}: {us:.1f} us, {2.0 * M * N * Kd / us / 1e6:.0f} TF, {tiles} tiles")
    for g in range(2):
        n = d[:, g, 4]
        per = d[:, g, :4] / n[:, None]
        loop = d[:, g, 5] / (n + 2)
        print(f"  group {g}: cycles/slot  read+issue{'+wait' if g else ''} {per[:, 0].mean():7.0f}  bar1 {per[:, 1].mean():7.0f}"
              f"  mfma{'' if g else '+wait'} {per[:, 2].mean():7.0f}  bar2 {per[:, 3].mean():7.0f}   loop/slot {loop.mean():7.0f}"
              f"  (min/max loop/slot over blocks {loop.min():.0f}/{loop.max():.0f})")
K.call("mms2ut_gemm_set_pp", -1)
