"""Isolated timings of the step's wide NT GEMM shapes under the current tile order / build (for L2
locality A/Bs: MMS2UT_GEMM_GROUP_M, MMS2UT_GEMM_PP, MMS2UT_LIB).  Random fp16 operands, warm, HIP
events over 20 launches per shape.  Under rocprofv3 --pmc each shape's launches are dispatches
with distinct grids (scripts/pmc_dispatch.py groups them).
usage: python scripts/gemm_l2_ab.py [reps]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
M = 10000
line = []
for name, N, Kd, epi in (("fc1_fwd", 3072, 768, "RELU_DROP"), ("qkv_fwd", 2304, 768, "F16"),
                         ("fc2_dgrad", 3072, 768, "RELU_DROP_BWD"), ("fc2_fwd", 768, 3072, "DROP_RESID"),
                         ("out_proj", 768, 768, "DROP_RESID"), ("qkv_dgrad", 768, 2304, "F16")):
    g = torch.Generator(device="cuda").manual_seed(N + Kd)
    x = (torch.randn(M, Kd, device="cuda", generator=g) * 0.5).half()
    W = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).half()
    b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
    aux = torch.randn(M, N, device="cuda", generator=g).half()
    out = torch.empty(M, N, dtype=torch.float16, device="cuda")
    e = getattr(K, "EPI_" + epi)
    ua = epi in ("DROP_RESID", "RELU_DROP_BWD")

    def run():
        K.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, epi=e, bias=b, aux=aux if ua else None, ldaux=N,
               p=0.1 if epi != "F16" else 0.0, seed=5, offset=0, ld_rng=N, fixup=False)
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    line.append(f"{name} {us:6.1f} us ({2.0 * M * N * Kd / us / 1e6:4.0f} TF)")
print("  ".join(line), flush=True)
