"""Weight-gradient shapes (dW[N_out, K_in] = dy[rows, N_out]^T x[rows, K_in], both operands
M/N-contiguous) on the grouped 128x128 kernel (mms2ut_wgrad_group, one problem or a whole layer)
and on plain mms2ut_gemm_f16 launches (whatever tile gemm_dispatch picks in the library under test:
MMS2UT_LIB).  Mean of 20 warm launches, HIP events, random fp16.
usage: python scripts/wgrad_ab.py [rows]"""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
layer = [("qkv", 2304, 768), ("out", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)]


def timeit(f, n=20):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = {}
ops = {}
for name, N, Kin in layer:
    dy = torch.randn(rows, N, device="cuda").half()
    x = torch.randn(rows, Kin, device="cuda").half()
    dW = torch.empty(N, Kin, device="cuda", dtype=torch.float16)
    db = torch.empty(N, device="cuda", dtype=torch.float16)
    ops[name] = (dy, x, dW, db)
    fl = 2.0 * rows * N * Kin
    us_g = timeit(lambda: K.wgrad_group([(dy, x, dW, db)], rows))
    us_p = timeit(lambda: K.gemm(dy, x, dW, N, Kin, rows, a_kc=False, b_kc=False, lda=N, ldb=Kin, ldc=Kin))
    res[name] = {"group_us": round(us_g, 1), "group_tf": round(fl / us_g / 1e6), "plain_us": round(us_p, 1),
                 "plain_tf": round(fl / us_p / 1e6)}
fl = sum(2.0 * rows * N * Kin for _, N, Kin in layer)
us = timeit(lambda: K.wgrad_group([ops[n] for n, _, _ in layer], rows))
res["layer grouped"] = {"us": round(us, 1), "tf": round(fl / us / 1e6)}
# many layers' worth of tiles in one product: M = 8 x 2304 stacked outputs
dy = torch.randn(rows, 8 * 2304, device="cuda").half()
x = torch.randn(rows, 768, device="cuda").half()
dW = torch.empty(8 * 2304, 768, device="cuda", dtype=torch.float16)
us = timeit(lambda: K.gemm(dy, x, dW, 8 * 2304, 768, rows, a_kc=False, b_kc=False, lda=8 * 2304, ldb=768, ldc=768))
res["plain 18432x768"] = {"us": round(us, 1), "tf": round(2.0 * rows * 8 * 2304 * 768 / us / 1e6)}
print(json.dumps(res))
