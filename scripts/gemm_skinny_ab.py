"""Short-M NT GEMM routes on the decoder's shapes (M = target tokens of a bench batch): the whole-K
small-tile kernel (default), split-K + fixup, and the unsplit 128x128 kernel.  Each route runs
REPS launches captured in one HIP graph (so host issue cost is out) and replayed; the table gives
GPU microseconds per GEMM (kernel + the gap to the next launch, both kernels for the fixup).

    python scripts/gemm_skinny_ab.py [M] [REPS]
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels

M = int(sys.argv[1]) if len(sys.argv) > 1 else 470
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 50
SHAPES = [("f16", 768, 768), ("relu_drop", 3072, 768), ("drop_resid", 768, 3072), ("f16", 2304, 768),
          ("relu_drop_bwd", 3072, 768), ("f16", 768, 2304), ("drop_resid", 768, 768), ("f16", 768, 3072),
          ("f16", 1536, 768), ("f16", 1536, 2560)]
ROUTES = (("skinny", 1, True), ("fixup", 0, True), ("unsplit", 0, False))


def run(name, N, Kd, fix):
    epi = getattr(K, "EPI_" + name.upper())
    x = run.x[:, :Kd]
    W = run.W[:N, :Kd]
    aux = run.aux[:, :N] if name in ("drop_resid", "relu_drop_bwd") else None
    p = 0.1 if name in ("relu_drop", "drop_resid", "relu_drop_bwd") else 0.0
    K.gemm(x, W, run.out[:, :N], M, N, Kd, lda=x.stride(0), ldb=W.stride(0), ldc=run.out.stride(0), epi=epi,
           bias=None if name == "relu_drop_bwd" else run.b[:N], aux=aux, ldaux=run.aux.stride(0), p=p, seed=5,
           offset=0, ld_rng=N, fixup=fix)


g = torch.Generator(device="cuda").manual_seed(0)
run.x = (torch.randn(M, 3072, device="cuda", generator=g) * 0.5).half()
run.W = (torch.randn(3072, 3072, device="cuda", generator=g) * 0.05).half()
run.b = torch.randn(3072, device="cuda", generator=g).half()
run.aux = torch.randn(M, 3072, device="cuda", generator=g).half()
run.out = torch.empty(M, 3072, device="cuda", dtype=torch.float16)
s = torch.cuda.Stream()
print(f"M = {M}, {REPS} launches per graph; us per GEMM (TF/s)")
print(f"{'epilogue':14s} {'N':>5s} {'K':>5s} " + " ".join(f"{r[0]:>16s}" for r in ROUTES))
try:
    for name, N, Kd in SHAPES:
        cells = []
        for route, skinny, fix in ROUTES:
            K.call("mms2ut_gemm_set_skinny", skinny)
            with torch.cuda.stream(s):
                run(name, N, Kd, fix)      # workspace allocation outside the capture
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=s):
                    for _ in range(REPS):
                        run(name, N, Kd, fix)
            graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                graph.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (3 * REPS)
            cells.append(f"{us:7.2f} ({2.0 * M * N * Kd / us / 1e6:5.0f})")
            del graph
        print(f"{name:14s} {N:5d} {Kd:5d} " + " ".join(f"{c:>16s}" for c in cells))
finally:
    K.call("mms2ut_gemm_set_skinny", 1)
