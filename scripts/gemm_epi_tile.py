"""128x128 vs 256x256 (gemm256p) tile on the fused-epilogue shapes of the FFN (N = 3072, K = 768):
relu+dropout forward (fc1) and relu-dropout backward (fc2 dgrad), interleaved rounds, random
operands.  usage: python scripts/gemm_epi_tile.py [M]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
M = int(sys.argv[1]) if len(sys.argv) > 1 else 10000


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


x = torch.randn(M, 768, device="cuda").half()
W1 = (0.05 * torch.randn(3072, 768, device="cuda")).half()
b1 = torch.randn(3072, device="cuda").half()
h = torch.empty(M, 3072, device="cuda", dtype=torch.float16)
dy = torch.randn(M, 768, device="cuda").half()
W2T = (0.05 * torch.randn(3072, 768, device="cuda")).half()   # fc2 W^T image [3072, 768]
dh = torch.empty(M, 3072, device="cuda", dtype=torch.float16)
cases = {
    "fc1 relu_drop": lambda: K.linear(x, W1, b1, out=h, epi=K.EPI_RELU_DROP, p=0.1, drop=(7, 0)),
    "fc1 f16+bias": lambda: K.linear(x, W1, b1, out=h),
    "fc2 dgrad relu_drop_bwd": lambda: K.gemm(dy, W2T, dh, M, 3072, 768, a_kc=True, b_kc=True, lda=768, ldb=768,
                                             ldc=3072, epi=K.EPI_RELU_DROP_BWD, aux=h, ldaux=3072, p=0.1),
}
res = {}
for rnd in range(3):
    for tile in ("1", "2"):
        os.environ["MMS2UT_GEMM_TILE"] = tile
        for name, fn in cases.items():
            res[(name, tile)] = min(res.get((name, tile), 1e9), t(fn))
fl = 2.0 * M * 3072 * 768
for name in cases:
    a, b = res[(name, "1")], res[(name, "2")]
    print(f"M={M} {name:26s} 128: {a:6.1f} us {fl / a / 1e6:5.0f} TF   256p: {b:6.1f} us {fl / b / 1e6:5.0f} TF", flush=True)
