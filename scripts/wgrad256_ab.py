"""TN weight-gradient GEMMs (dW[M, N] = dy[rows, M]^T x[rows, N], both operands M/N-contiguous) on
the 128x128 grouped kernel (mms2ut_wgrad_group, one problem) and on the 256x256 kernel
(MMS2UT_GEMM_256=1 forces it through mms2ut_gemm_f16).  usage: python scripts/wgrad256_ab.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels


def timeit(fn, reps=10):
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


for M, N, R in ((4096, 4096, 10000), (3072, 768, 10000), (2304, 768, 10000), (768, 3072, 10000), (768, 768, 10000),
                (3072, 3072, 10000)):
    g = torch.Generator(device="cuda").manual_seed(M + N)
    dy = (torch.randn(R, M, device="cuda", generator=g) * 0.1).half()
    x = (torch.randn(R, N, device="cuda", generator=g) * 0.1).half()
    dW = torch.empty(M, N, device="cuda", dtype=torch.float16)
    def grouped():
        K.wgrad_group([(dy, x, dW, None)], R)
    def t256():
        K.gemm(dy, x, dW, M, N, R, a_kc=False, b_kc=False, lda=M, ldb=N, ldc=N, epi=K.EPI_F16, fixup=False)
    tg = timeit(grouped)
    ref = dW.clone()
    t2 = timeit(t256)
    rel = ((dW.float() - ref.float()).norm() / ref.float().norm()).item()
    fl = 2.0 * M * N * R
    print(f"dW {M:5d}x{N:5d} rows {R}: grouped128 {tg:7.1f} us ({fl / tg / 1e6:5.0f} TF)   "
          f"gemm{'256' if os.environ.get('MMS2UT_GEMM_256') == '1' else '128'} {t2:7.1f} us ({fl / t2 / 1e6:5.0f} TF)  rel {rel:.1e}")
