"""NT GEMM outputs of the tall / 128x128 routes under step-like dropout streams (library under test:
MMS2UT_LIB): large and odd counter offsets, several seeds, the bench's ragged row counts, alpha != 1
with a bias, and overflowing accumulators.  Compare two dumps with scripts/wgrad_bits.py cmp.
usage: python scripts/gemm_bits2.py OUT.npz"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
out = {}
for M in (9607, 11003, 7589, 2000):
    for N, Kd in ((3072, 768), (768, 768), (2304, 768), (768, 3072), (1004, 768)):
        g = torch.Generator(device="cuda").manual_seed(M + 3 * N + Kd)
        x = (torch.randn(M, Kd, device="cuda", generator=g) * 0.5).half()
        W = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).half()
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
        key = f"M{M}_N{N}_K{Kd}"
        for oi, off in enumerate((0, 7, (1 << 33) - 12345678, 123456789012, (1 << 32) + 3)):
            seed = 1000 + oi * 7919
            out[f"{key}_relu_o{oi}"] = K.linear(x, W, b, epi=K.EPI_RELU_DROP, p=0.1, drop=(seed, off)).cpu().numpy()
        out[key + "_plain_nobias"] = K.linear(x, W).cpu().numpy()
        big = (x * 60).half()
        out[key + "_overflow"] = K.linear(big, W * 40, b).cpu().numpy()
        out[key + "_relu_overflow"] = K.linear(big, W * 40, b, epi=K.EPI_RELU_DROP, p=0.1, drop=(5, 99)).cpu().numpy()
np.savez(sys.argv[1], **out)
print("dumped", len(out))
