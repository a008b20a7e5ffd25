"""In-step vs isolated GEMM time per launch shape.

Reads a roofline-pass dump of bench.py (MMS2UT_GEMM_DUMP=path.npz) and re-times every distinct
(A/B layout, M, N, K, split, epilogue) isolated and warm (random operands, 20 back-to-back calls,
plain fp16 / fp32-slab epilogue), so the table separates what the shape costs from what the step
adds (cold operands, fused epilogues, stream contention).

    python scripts/gemm_instep.py path.npz
"""
import importlib
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels

z = np.load(sys.argv[1])
steps = int(z["steps"])
rows = defaultdict(lambda: [0, 0.0, 0.0])
for ms, fl, c, (M, N, Kd, nz) in zip(z["ms"], z["flops"], z["cls"], z["mnk"]):
    c = int(c)
    if c & 256:
        continue  # batched attention products: not re-timed
    key = (c & 1, (c >> 1) & 1, (c >> 2) & 63, int(M), int(N), int(Kd), int(nz))
    r = rows[key]
    r[0] += 1
    r[1] += float(ms)
    r[2] += float(fl)


def iso(a_kc, b_kc, epi, m, n, k, s, reps=20):
    A = (torch.rand(m, k, device="cuda") if a_kc else torch.rand(k, m, device="cuda")).sub_(0.5).half()
    B = (torch.rand(n, k, device="cuda") if b_kc else torch.rand(k, n, device="cuda")).sub_(0.5).half()
    f32 = epi == K.EPI_F32
    C = torch.empty((s if f32 else 1) * m, n, dtype=torch.float32 if f32 else torch.float16, device="cuda")

    def call():
        K.gemm(A, B, C, m, n, k, a_kc=bool(a_kc), b_kc=bool(b_kc), lda=A.stride(0), ldb=B.stride(0), ldc=n,
               epi=K.EPI_F32 if f32 else K.EPI_F16, splitk=s if f32 else 1, sCsplit=m * n)
    call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


tot_step = sum(r[1] for r in rows.values()) / steps
tot_iso = 0.0
print(f"{'layout':6s} {'epi':>3s} {'M':>6s} {'N':>5s} {'K':>6s} {'nz':>3s} {'n/st':>5s} {'step us':>8s} {'TF':>5s} "
      f"{'iso us':>8s} {'TF':>5s} {'step/iso':>8s}")
for key, (n, ms, fl) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
    a_kc, b_kc, epi, m, nn, k, nz = key
    per = ms / n * 1e3
    try:
        t = iso(a_kc, b_kc, epi, m, nn, k, nz) * 1e3
    except Exception as e:  # a shape the plain path cannot replay
        print("skip", key, e)
        continue
    tot_iso += t * n / steps / 1e3
    lay = ("K" if a_kc else "M") + ("K" if b_kc else "N")
    print(f"{lay:6s} {epi:3d} {m:6d} {nn:5d} {k:6d} {nz:3d} {n / steps:5.1f} {per:8.1f} {fl / n / per / 1e6:5.0f} "
          f"{t:8.1f} {fl / n / t / 1e6:5.0f} {per / t:8.2f}", flush=True)
print(f"total in-step {tot_step:.2f} ms/step, isolated {tot_iso:.2f} ms/step")
