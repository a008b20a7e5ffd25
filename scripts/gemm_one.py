"""Run one GEMM shape repeatedly (for rocprofv3 --pmc on a single kernel).
usage: python scripts/gemm_one.py M N K a_kc b_kc [splitk] [reps]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels

M, N, Kd, akc, bkc = (int(x) for x in sys.argv[1:6])
s = int(sys.argv[6]) if len(sys.argv) > 6 else 1
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 10
A = torch.randn(M, Kd, device="cuda").half() if akc else torch.randn(Kd, M, device="cuda").half()
B = torch.randn(N, Kd, device="cuda").half() if bkc else torch.randn(Kd, N, device="cuda").half()
C = torch.empty(s, M, N, dtype=torch.float32, device="cuda") if s > 1 else torch.empty(M, N, dtype=torch.float16, device="cuda")
for _ in range(reps):
    K.gemm(A, B, C, M, N, Kd, a_kc=bool(akc), b_kc=bool(bkc), lda=A.stride(0), ldb=B.stride(0), ldc=N,
           epi=K.EPI_F32 if s > 1 else K.EPI_F16, splitk=s, sCsplit=M * N)
torch.cuda.synchronize()
