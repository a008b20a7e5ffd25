"""Vendor-library calibration: torch.mm (hipBLASLt / rocBLAS) fp16 on the training step's GEMM
shapes, random operands, warm, 20 back-to-back calls.  What a tuned library reaches on exactly
these shapes (not a product path).

    python scripts/blas_ref.py [M]
"""
import sys

import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
SHAPES = [("qkv fwd", M, 2304, 768), ("fc1 fwd", M, 3072, 768), ("fc2 fwd", M, 768, 3072),
          ("out fwd", M, 768, 768), ("qkv dgrad", M, 768, 2304), ("wgrad 3072x768", 3072, 768, M),
          ("square 4096", 4096, 4096, 4096), ("square 8192", 8192, 8192, 8192)]
for name, m, n, k in SHAPES:
    a = torch.rand(m, k, device="cuda").sub_(0.5).half()
    b = torch.rand(n, k, device="cuda").sub_(0.5).half()
    for tb in (True,):
        bb = b.t() if tb else b
        for _ in range(3):
            torch.mm(a, bb)
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                torch.mm(a, bb)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 20)
        print(f"{name:16s} M={m:6d} N={n:5d} K={k:6d}  {best * 1e3:7.1f} us  {2.0 * m * n * k / best / 1e9:6.0f} TF/s",
              flush=True)
