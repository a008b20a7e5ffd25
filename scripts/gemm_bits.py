"""NT GEMM outputs and isolated times on the step's shapes for the library under test (MMS2UT_LIB):
dump seeded linear() results (plain, ReLU+dropout, dropout+residual epilogues) to an .npz and print
us / TF/s per shape; compare two dumps with scripts/wgrad_bits.py cmp.
usage: python scripts/gemm_bits.py OUT.npz"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels


def timeit(fn, reps=20):
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


out, times = {}, {}
for M in (10000, 12000, 777):
    for N, Kd in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        g = torch.Generator(device="cuda").manual_seed(M * 7 + N + Kd)
        x = (torch.randn(M, Kd, device="cuda", generator=g) * 0.5).half()
        W = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).half()
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
        res = torch.randn(M, N, device="cuda", generator=g).half()
        key = f"M{M}_N{N}_K{Kd}"
        out[key + "_plain"] = K.linear(x, W, b).cpu().numpy()
        out[key + "_relu"] = K.linear(x, W, b, epi=K.EPI_RELU_DROP, p=0.1, drop=(1234, 0)).cpu().numpy()
        out[key + "_resid"] = K.linear(x, W, b, epi=K.EPI_DROP_RESID, aux=res, p=0.1, drop=(99, 0)).cpu().numpy()
        if M != 777:
            us = timeit(lambda: K.linear(x, W, b))
            times[key] = {"us": round(us, 1), "tf": round(2.0 * M * N * Kd / us / 1e6)}
np.savez(sys.argv[1], **out)
print(json.dumps(times))
