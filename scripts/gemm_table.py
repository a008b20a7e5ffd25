"""Summarise a bench roofline-pass GEMM dump (MMS2UT_GEMM_DUMP=path.npz python bench.py ...):
per (class, M-bucket, N, K, epilogue) the launches per step, time per step and TF/s.

    python scripts/gemm_table.py path.npz
"""
import sys
from collections import defaultdict

import numpy as np

EPI = {0: "f16", 1: "relu_drop", 2: "drop_resid", 3: "f32", 4: "gate", 5: "relu_drop_bwd", 6: "f16_acc", 7: "gelu_drop",
       8: "gelu_drop_bwd"}
z = np.load(sys.argv[1])
steps = int(z["steps"])
rows = defaultdict(lambda: [0, 0.0, 0.0])
for ms, fl, c, (M, N, K, nz) in zip(z["ms"], z["flops"], z["cls"], z["mnk"]):
    kind = "batched" if c & 256 else ("TN" if not (c & 3) else ("NT" if (c & 3) == 3 else "NN"))
    kind += "/sm" if c & 2048 else ""   # short-M kernel (csrc/gemm_skinny.h)
    key = (kind, EPI[(int(c) >> 2) & 63], N, K, nz, M // 2000 * 2000)
    r = rows[key]
    r[0] += 1
    r[1] += float(ms)
    r[2] += float(fl)
tot = sum(r[1] for r in rows.values())
print(f"total GEMM {tot / steps:.2f} ms/step")
for k, (n, ms, fl) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[0]:7s} {k[1]:13s} N={k[2]:5d} K={k[3]:6d} nz={k[4]:3d} M~{k[5]:6d}: {n / steps:5.1f}/step "
          f"{ms / steps * 1e3:7.1f} us/step {fl / ms / 1e9:6.0f} TF/s")
