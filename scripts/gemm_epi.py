"""Isolated GEMM time per epilogue on the step's shapes (random operands): how much of the
in-step GEMM time the fused epilogues (dropout hash, residual read) cost.

    python scripts/gemm_epi.py [M]
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels
M = int(sys.argv[1]) if len(sys.argv) > 1 else 7600


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for n, k in ((3072, 768), (768, 3072), (768, 768), (2304, 768)):
    x = torch.randn(M, k, device="cuda").half()
    W = torch.randn(n, k, device="cuda").half() * 0.05
    b = torch.randn(n, device="cuda").half()
    aux = torch.randn(M, n, device="cuda").half()
    out = torch.empty(M, n, device="cuda", dtype=torch.float16)
    fl = 2.0 * M * n * k
    res = {}
    for rnd in range(2):
        for name, kw in (("f16", {}), ("bias", {"bias": b}),
                         ("relu_drop", {"bias": b, "epi": K.EPI_RELU_DROP, "p": 0.1, "drop": (7, 0)}),
                         ("relu_nodrop", {"bias": b, "epi": K.EPI_RELU_DROP}),
                         ("drop_resid", {"bias": b, "epi": K.EPI_DROP_RESID, "aux": aux, "p": 0.1, "drop": (7, 0)}),
                         ("resid_nodrop", {"bias": b, "epi": K.EPI_DROP_RESID, "aux": aux})):
            kw = dict(kw)
            bias = kw.pop("bias", None)
            t = timeit(lambda: K.linear(x, W, bias, out=out, **kw))
            res[name] = min(res.get(name, 1e9), t)
    print(f"M={M} N={n:5d} K={k:5d} " + "  ".join(f"{a}: {v*1e3:6.1f}us {fl/v/1e9:4.0f}TF" for a, v in res.items()),
          flush=True)
