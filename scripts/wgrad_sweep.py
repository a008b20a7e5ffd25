"""Weight-gradient GEMM (both operands M/N-contiguous, reduction over the token rows) on the step's
shapes: 128x128 vs 256x256 ring tiles at several split-K counts (time of GEMM alone + the fp32
slab reduction it implies).  usage: python scripts/wgrad_sweep.py [tokens]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
T = int(sys.argv[1]) if len(sys.argv) > 1 else 8704
SHAPES = [("fc1 3072x768", 3072, 768), ("fc2 768x3072", 768, 3072), ("qkv 2304x768", 2304, 768),
          ("out 768x768", 768, 768), ("xkv 9216x768", 9216, 768)]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, n_out, k_in in SHAPES:
    dy = torch.randn(T, n_out, device="cuda").half()
    x = torch.randn(T, k_in, device="cuda").half()
    ref = dy.float().t() @ x.float()
    line = f"{name:14s}"
    for tile in ("1", "2"):
        os.environ["MMS2UT_GEMM_TILE"] = tile
        for s in (1, 2, 4, 6, 8, 12):
            slab = torch.empty(s, n_out, k_in, dtype=torch.float32, device="cuda")
            dW = torch.empty(n_out, k_in, dtype=torch.float16, device="cuda")

            def g():
                K.gemm(dy, x, slab, n_out, k_in, T, a_kc=False, b_kc=False, lda=n_out, ldb=k_in, ldc=k_in,
                       epi=K.EPI_F32, splitk=s, sCsplit=n_out * k_in)

            def r():
                K.call("mms2ut_splitk_reduce", slab.data_ptr(), s, n_out * k_in, n_out, k_in, dW.data_ptr(), k_in,
                       1, 1.0, K._s())
            tg, tr = timed(g), timed(r)
            g(); r(); torch.cuda.synchronize()
            err = ((dW.float() - ref).norm() / ref.norm()).item()
            fl = 2.0 * n_out * k_in * T
            line += f" | t{tile} s{s:2d} {tg:6.1f}+{tr:5.1f}us {fl / (tg + tr) / 1e6:4.0f}TF" + ("" if err < 3e-3 else " BAD")
    print(line, flush=True)
