"""Warm vs cold-cache GEMM time on the step's shapes: the same operands re-used (L2 / MALL hot,
what the retired scripts/gemm_shapes.py measured) vs a rotation over operand sets larger than the 256 MiB
MALL with a 512 MiB sweep between calls (what the training step sees).

    python scripts/gemm_cold.py [M]
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels
M = int(sys.argv[1]) if len(sys.argv) > 1 else 11000
sweep = torch.empty(256 * 1024 * 1024, dtype=torch.float16, device="cuda")


def run(n, k, epi, cold, reps=12):
    sets = []
    for i in range(4 if cold else 1):
        x = torch.randn(M, k, device="cuda").half()
        W = (torch.randn(n, k, device="cuda") * 0.05).half()
        aux = torch.randn(M, n, device="cuda").half()
        out = torch.empty(M, n, device="cuda", dtype=torch.float16)
        sets.append((x, W, aux, out))
    b = torch.randn(n, device="cuda").half()
    ts = []
    for r in range(reps):
        x, W, aux, out = sets[r % len(sets)]
        if cold:
            sweep.add_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        kw = {}
        if epi == "relu_drop":
            kw = dict(epi=K.EPI_RELU_DROP, p=0.1, drop=(7, 0))
        elif epi == "drop_resid":
            kw = dict(epi=K.EPI_DROP_RESID, aux=aux, p=0.1, drop=(7, 0))
        e0.record()
        K.linear(x, W, b, out=out, **kw)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts = sorted(ts[2:])
    return ts[len(ts) // 2]


for n, k, epi in ((3072, 768, "relu_drop"), (768, 3072, "drop_resid"), (768, 768, "f16"), (2304, 768, "f16"),
                  (768, 768, "drop_resid")):
    fl = 2.0 * M * n * k
    w, c = run(n, k, epi, False), run(n, k, epi, True)
    print(f"M={M} N={n:5d} K={k:5d} {epi:10s} warm {w:6.1f} us {fl / w / 1e6:5.0f} TF   cold {c:6.1f} us "
          f"{fl / c / 1e6:5.0f} TF", flush=True)
