"""Per-workgroup timing of single GEMM launches (in-kernel s_memrealtime stamps, mms2ut_profile_stamps):
launch span, the spread of workgroup start times (dispatch) and the workgroup durations.

    python scripts/gemm_blocks.py M N K [epi] [skinny 0/1] [fixup 0/1]
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels

M, N, Kd = (int(v) for v in sys.argv[1:4])
epi = getattr(K, "EPI_" + (sys.argv[4].upper() if len(sys.argv) > 4 else "F16"))
skinny = int(sys.argv[5]) if len(sys.argv) > 5 else 1
fix = bool(int(sys.argv[6])) if len(sys.argv) > 6 else True
K.call("mms2ut_gemm_set_skinny", skinny)
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, Kd, device="cuda", generator=g) * 0.5).half()
W = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).half()
b = torch.randn(N, device="cuda", generator=g).half()
out = torch.empty(M, N, device="cuda", dtype=torch.float16)
khz = ctypes.c_int()
K.call("mms2ut_wallclock_khz", ctypes.byref(khz))
tick_us = 1e3 / khz.value
for it in range(4):
    stamps = torch.zeros(2 * 200_000, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    K.gemm_profile_begin(10)
    K.gemm_profile_stamps(stamps)
    K.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, epi=epi, bias=b, fixup=fix)
    torch.cuda.synchronize()
    _, n, _, _ = K.gemm_profile_end()
    fl = np.zeros((n, 2), np.int64)
    K.call("mms2ut_profile_blocks", fl.ctypes.data, int(n))
    st = stamps.view(-1, 2).cpu().numpy()[fl[0, 0]:fl[0, 1]]
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    s = (st[:, 0] - t0) * tick_us
    e = (st[:, 1] - t0) * tick_us
    d = e - s
    print(f"run {it}: {len(st)} workgroups, span {e.max():6.2f} us; starts 0..{s.max():5.2f} us "
          f"(median {np.median(s):5.2f}); durations min {d.min():5.2f} median {np.median(d):5.2f} max {d.max():5.2f} us")
K.call("mms2ut_gemm_set_skinny", 1)
