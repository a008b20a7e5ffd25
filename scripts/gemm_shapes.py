"""Per-shape GEMM throughput on the training step's shapes: the library's default dispatch, the
forced 128x128 and 256x256 kernels, and hipBLASLt through torch.matmul on the same operands
(reference point only).  Weight gradients include their split-K slab reduction, as in the step.
Random operands; interleaved rounds in one process (cdna guide §5.4 rule 24).

    python scripts/gemm_shapes.py [M]
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels

M = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
FWD = [("qkv", 2304, 768), ("out/q", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072),
       ("cross-kv x6", 9216, 768), ("gate", 768, 1536)]
WGRAD = [("wg qkv", 2304, 768), ("wg out", 768, 768), ("wg fc1", 3072, 768), ("wg fc2", 768, 3072),
         ("wg cross-kv", 9216, 768)]


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


def fwd_case(name, n, k):
    x = torch.randn(M, k, device="cuda").half()
    W = torch.randn(n, k, device="cuda").half()
    out = torch.empty(M, n, device="cuda", dtype=torch.float16)
    fl = 2.0 * M * n * k
    res = {}
    for rnd in range(2):
        for tile in ("auto", "128", "256"):
            if tile == "auto":
                os.environ.pop("MMS2UT_GEMM_TILE", None)
            else:
                os.environ["MMS2UT_GEMM_TILE"] = tile
            t = timeit(lambda: K.linear(x, W, out=out))
            res[tile] = min(res.get(tile, 1e9), t)
        os.environ.pop("MMS2UT_GEMM_TILE", None)
        t = timeit(lambda: torch.matmul(x, W.t()))
        res["torch"] = min(res.get("torch", 1e9), t)
    print(f"{name:12s} M={M} N={n:5d} K={k:5d} " + "  ".join(
        f"{k_}: {v*1e3:6.1f}us {fl/v/1e9:5.0f}TF" for k_, v in res.items()), flush=True)


def wgrad_case(name, n, k):
    dy = torch.randn(M, n, device="cuda").half()
    x = torch.randn(M, k, device="cuda").half()
    dW = torch.empty(n, k, device="cuda", dtype=torch.float16)
    db = torch.empty(n, device="cuda", dtype=torch.float16)
    fl = 2.0 * M * n * k
    res = {}
    for rnd in range(2):
        res["lib"] = min(res.get("lib", 1e9), timeit(lambda: K.linear_wgrad(dy, x, dW, db=db, side=False)))
        res["torch"] = min(res.get("torch", 1e9), timeit(lambda: torch.matmul(dy.t(), x)))
    print(f"{name:12s} M={n:5d} N={k:5d} K={M} " + "  ".join(
        f"{k_}: {v*1e3:6.1f}us {fl/v/1e9:5.0f}TF" for k_, v in res.items()), flush=True)


if __name__ == "__main__":
    for c in FWD:
        fwd_case(*c)
    for c in WGRAD:
        wgrad_case(*c)
