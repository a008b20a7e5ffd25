"""Isolated timings of the HBM-bound kernels on the training step's shapes (achieved GB/s of
algorithmic bytes).  Usage: python scripts/ops_bench.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def report(name, us, nbytes):
    print(f"{name:34s} {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s  ({nbytes / 1e6:.1f} MB)", flush=True)


def main():
    dev = "cuda"
    R, D, F = 9600, 768, 3072
    x = torch.randn(R, D, device=dev).half()
    g = torch.ones(D, device=dev).half()
    b = torch.zeros(D, device=dev).half()
    y, mean, rstd = K.layernorm(x, g, b)
    report("layernorm_fwd 9600x768", timeit(lambda: K.layernorm(x, g, b)), 2 * R * D * 2)
    dy = torch.randn(R, D, device=dev).half()
    dres = torch.randn(R, D, device=dev).half()
    dgb = torch.empty(2 * D, dtype=torch.float16, device=dev)
    report("layernorm_bwd (+dres)", timeit(lambda: K.layernorm_bwd(dy, x, g, mean, rstd, dgb, dres=dres)),
           4 * R * D * 2)
    report("layernorm_bwd (+dres, emit drop)",
           timeit(lambda: K.layernorm_bwd(dy, x, g, mean, rstd, dgb, dres=dres, emit=(0.1, (1, 0)))),
           5 * R * D * 2)
    Ri = 80 * 577
    xi = torch.randn(Ri, D, device=dev).half()
    _, mi, ri = K.layernorm(xi, g, b)
    dyi = torch.randn(Ri, D, device=dev).half()
    report("layernorm_bwd params-only 46k", timeit(lambda: K.layernorm_bwd(dyi, xi, g, mi, ri, dgb, want_dx=False)),
           2 * Ri * D * 2)
    dF = torch.randn(R, F, device=dev).half()
    db = torch.empty(F, dtype=torch.float16, device=dev)
    report("bias_grad 9600x3072", timeit(lambda: K.bias_grad(dF, db, side=False)), R * F * 2)
    report("bias_grad 9600x768", timeit(lambda: K.bias_grad(dy, db[:D], side=False)), R * D * 2)
    for s in (4, 7, 14):
        slabs = torch.randn(s, F, D, device=dev)
        out = torch.empty(F, D, dtype=torch.float16, device=dev)
        report(f"splitk_reduce s={s} 3072x768",
               timeit(lambda: K.call("mms2ut_splitk_reduce", slabs.data_ptr(), s, F * D, F, D, out.data_ptr(),
                                     D, 1, 1.0, K._s())), s * F * D * 4 + F * D * 2)
    out = torch.empty_like(dy)
    report("dropout 9600x768", timeit(lambda: K.dropout(dy, 0.1, (1, 0), out=out)), 2 * R * D * 2)
    n = 164_000_000
    p16 = torch.randn(n, device=dev).half()
    g16 = torch.randn(n, device=dev).half() * 1e-3
    master = p16.float()
    m1 = torch.zeros(n, device=dev)
    m2 = torch.zeros(n, device=dev)
    ost = torch.zeros(16, device=dev)
    ost[K.OST_MULT] = 1.0
    ost[K.OST_CLIP_COEF] = 1.0
    ost[K.OST_STEP_SIZE] = 1e-4
    report("adam 164M", timeit(lambda: K.adam(p16, g16, master, m1, m2, ost, 0.9, 0.98, 1e-8, 0.0), reps=5),
           n * (2 + 2 + 12 + 12))
    # attention backward prep: rowsum(dO * O) per head
    B, T, H = 80, 120, 8
    O = torch.randn(B * T, D, device=dev).half()
    dO = torch.randn(B * T, D, device=dev).half()
    Dd = torch.empty(B * H * T, device=dev)
    print("(attention prep timed inside mha_bwd; see rocprof)")


if __name__ == "__main__":
    main()
