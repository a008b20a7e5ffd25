"""A/B of the HIP GEMM tile paths (128x128 LDS-DMA vs 256x256 ring) on the training step's shapes:
correctness against torch fp32 and interleaved timing in one process.  Random operands.

    python scripts/gemm_ab.py [M]
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels

M = int(sys.argv[1]) if len(sys.argv) > 1 else 8704
SHAPES = [  # name, M, N, K, a_kc, b_kc, splitk
    ("qkv fwd", M, 2304, 768, True, True, 1),
    ("fc1 fwd", M, 3072, 768, True, True, 1),
    ("fc2 fwd", M, 768, 3072, True, True, 1),
    ("out fwd", M, 768, 768, True, True, 1),
    ("fc2 dgrad", M, 3072, 768, True, False, 1),
    ("fc1 dgrad", M, 768, 3072, True, False, 1),
    ("qkv dgrad", M, 768, 2304, True, False, 1),
    ("wgrad 3072x768 s8", 3072, 768, M, False, False, 8),
    ("wgrad 3072x768 s2", 3072, 768, M, False, False, 2),
    ("wgrad 2304x768 s4", 2304, 768, M, False, False, 4),
    ("wgrad 768x768 s8", 768, 768, M, False, False, 8),
    ("conv2 fwd", M, 1536, 2560, True, True, 1),
    ("square 4096", 4096, 4096, 4096, True, True, 1),
    ("square 8192", 8192, 8192, 8192, True, True, 1),
]
PATHS = {"128": {"MMS2UT_GEMM_TILE": "1"}, "256": {"MMS2UT_GEMM_TILE": "2", "MMS2UT_GEMM256": "0"},
         "256p4": {"MMS2UT_GEMM_TILE": "2", "MMS2UT_GEMM256": "4"}, "256p5": {"MMS2UT_GEMM_TILE": "2", "MMS2UT_GEMM256": "5"}}


def run(name, m, n, k, a_kc, b_kc, s, reps=20):
    torch.manual_seed(0)
    A = torch.rand(m, k, device="cuda").sub_(0.5).half() if a_kc else torch.rand(k, m, device="cuda").sub_(0.5).half()
    B = torch.rand(n, k, device="cuda").sub_(0.5).half() if b_kc else torch.rand(k, n, device="cuda").sub_(0.5).half()
    Af = (A if a_kc else A.t()).float()
    Bf = (B if b_kc else B.t()).float()
    ref = Af @ Bf.t()
    if s > 1:
        C = torch.empty(s, m, n, dtype=torch.float32, device="cuda")
        epi = K.EPI_F32
    else:
        C = torch.empty(m, n, dtype=torch.float16, device="cuda")
        epi = K.EPI_F16

    def call():
        K.gemm(A, B, C, m, n, k, a_kc=a_kc, b_kc=b_kc, lda=A.stride(0), ldb=B.stride(0), ldc=n,
               epi=epi, splitk=s, sCsplit=m * n)

    res, err = {}, {}
    for rnd in range(3):
        for tag, env in PATHS.items():
            os.environ.update(env)
            C.zero_()
            call()
            torch.cuda.synchronize()
            out = C.float().sum(0) if s > 1 else C.float()
            err[tag] = ((out - ref).norm() / ref.norm()).item()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            res[tag] = min(res.get(tag, 1e9), e0.elapsed_time(e1) / reps)
    os.environ.pop("MMS2UT_GEMM_TILE", None)
    fl = 2.0 * m * n * k
    line = f"{name:20s} M={m:6d} N={n:5d} K={k:6d}"
    for tag in PATHS:
        line += f" | {tag} {res[tag]*1e3:6.1f}us {fl/res[tag]/1e9:5.0f}TF {err[tag]:.0e}"
    print(line, flush=True)
    bad = [t for t in PATHS if not err[t] < 2e-3]
    return bad


def epilogue_check(m=1000, n=768, k=768):
    """Every fused epilogue of the 256 path against the 128 path (same rounding points)."""
    x = torch.randn(m, k, device="cuda").half()
    W = torch.randn(n, k, device="cuda").half() * 0.05
    b = torch.randn(n, device="cuda").half()
    res = torch.randn(m, n, device="cuda").half()
    aux2 = torch.randn(m, 2 * n, device="cuda").half()
    cases = [("bias", dict(epi=K.EPI_F16, bias=b)),
             ("resid p=.1", dict(epi=K.EPI_DROP_RESID, bias=b, aux=res, p=0.1, drop=(7, 512))),
             ("relu p=.1", dict(epi=K.EPI_RELU_DROP, bias=b, p=0.1, drop=(7, 512))),
             ("gate", dict(epi=K.EPI_GATE, bias=b, aux=aux2))]
    bad = []
    for name, kw in cases:
        outs = {}
        for tag, env in PATHS.items():
            os.environ.update(env)
            out2 = torch.zeros(m, n, dtype=torch.float16, device="cuda") if name == "gate" else None
            o = K.linear(x, W, out2=out2, **kw)
            outs[tag] = (o.float(), None if out2 is None else out2.float())
        os.environ.pop("MMS2UT_GEMM_TILE", None)
        d = 0.0
        for t in PATHS:
            d = max(d, (outs["128"][0] - outs[t][0]).abs().max().item())
            if outs["128"][1] is not None:
                d = max(d, (outs["128"][1] - outs[t][1]).abs().max().item())
        print(f"epilogue {name:12s} max|t128-other| = {d:.3e}", flush=True)
        if not d < 2e-2:
            bad.append(name)
    return bad


if __name__ == "__main__":
    bad = []
    bad += epilogue_check()
    for sh in SHAPES:
        bad += [(sh[0], t) for t in run(*sh)]
    print("FAILURES:", bad if bad else "none")
