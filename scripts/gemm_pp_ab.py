"""Isolated A/B of the NT GEMM kernels on the training step's shapes: the 128x128 LDS-DMA kernel
(mode 0) against the ping-pong 256-column kernel at each tile height (128 / 192 / 256) and the
automatic choice (-1).  Random fp16 operands, warm, HIP events over 20 launches; prints us and
TF/s per (shape, epilogue, mode) and checks every mode bit-identical to mode 0.
usage: python scripts/gemm_pp_ab.py [OUT.json]"""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
MODES = (0, 128, 192, 256, -1)


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


res = []
shapes = [(N, Kd, epi) for N, Kd, epi in ((3072, 768, "RELU_DROP"), (2304, 768, "F16"), (3072, 768, "RELU_DROP_BWD"),
                                          (768, 768, "DROP_RESID"), (768, 3072, "DROP_RESID"), (768, 3072, "F16"),
                                          (768, 2304, "F16"), (768, 768, "F16"))]
for M in (7680, 10000, 12000):
    for N, Kd, name in shapes:
        g = torch.Generator(device="cuda").manual_seed(M + N + Kd)
        x = (torch.randn(M, Kd, device="cuda", generator=g) * 0.5).half()
        W = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).half()
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
        aux = torch.randn(M, N, device="cuda", generator=g).half()
        out = torch.empty(M, N, dtype=torch.float16, device="cuda")
        epi = getattr(K, "EPI_" + name)
        use_aux = name in ("DROP_RESID", "RELU_DROP_BWD")
        p = 0.1 if name != "F16" else 0.0

        def run():
            K.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, epi=epi, bias=b, aux=aux if use_aux else None,
                   ldaux=N, p=p, seed=5, offset=0, ld_rng=N, fixup=False)
        row = {"M": M, "N": N, "K": Kd, "epi": name}
        ref = None
        for mode in MODES:
            K.call("mms2ut_gemm_set_pp", mode)
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            elif not torch.equal(out.view(torch.int16), ref.view(torch.int16)):
                row[f"bits_{mode}"] = "DIFFER"
            us = timeit(run)
            row[str(mode)] = round(us, 1)
        K.call("mms2ut_gemm_set_pp", -1)
        fl = 2.0 * M * N * Kd
        best = min(MODES[1:4], key=lambda m: row[str(m)])
        print(f"M={M:5d} N={N:4d} K={Kd:4d} {name:13s} 128sq {row['0']:7.1f} us ({fl / row['0'] / 1e6:5.0f} TF)  "
              + "  ".join(f"pp{m} {row[str(m)]:7.1f}" for m in MODES[1:4])
              + f"  auto {row['-1']:7.1f} ({fl / row['-1'] / 1e6:5.0f} TF)  best pp{best} {fl / row[str(best)] / 1e6:5.0f} TF"
              + ("  " + " ".join(k for k in row if k.startswith("bits")) if any(k.startswith("bits") for k in row) else ""),
              flush=True)
        res.append(row)
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
