"""Phase timing of the fused attention backward (diagnostic build, scripts/build_diag.sh): per
chunk, the cycles (s_memtime) spent waiting at the phase-1 barrier, in phase 1 (LDS stores of the
staged rows + D + next loads issued), phase 2 (dK/dV/dS), the phase-3 barrier and phase 3 (dQ),
median over the first 64 blocks.

    MMS2UT_LIB=multimodal-s2ut_amd/lib/libmms2ut_hip_diag.so python scripts/attn_phases.py B T [causal]
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels
lib = ctypes.CDLL(mm._lib.LIB_PATH)
lib.mms2ut_diag_attn_phases.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]

B, T = int(sys.argv[1]), int(sys.argv[2])
causal = len(sys.argv) > 3 and sys.argv[3] == "1"
H, d, p = 8, 768, float(os.environ.get("ATTN_P", "0.1"))
hd = d // H
dev = "cuda"
qkv = torch.randn(B * T, 3 * d, device=dev).half()
O = torch.empty(B * T, d, dtype=torch.float16, device=dev)
lens = torch.full((B,), T, dtype=torch.int32, device=dev)
lse = torch.empty(B * H * T, dtype=torch.float32, device=dev)
sq = T * 3 * d
args = (qkv, qkv[:, d:], qkv[:, 2 * d:], O, 3 * d, 3 * d, 3 * d, d, B, H, T, T, hd, hd ** -0.5)
K.call("mms2ut_mha_varlen_fwd", K._attn_args(*args, lens, causal, p, (3, 0), lse, sq=sq, sk=sq, sv=sq, so=T * d),
       K._s())
dO = torch.randn(B * T, d, device=dev).half()
dqkv = torch.empty_like(qkv)
Dd = torch.empty(B * H * T, dtype=torch.float32, device=dev)


def bwd():
    a = K._attn_args(*args, lens, causal, p, (3, 0), lse, sq=sq, sk=sq, sv=sq, so=T * d)
    K.call("mms2ut_mha_varlen_bwd", a, dO.data_ptr(), d, T * d, Dd.data_ptr(), dqkv.data_ptr(), 3 * d, sq,
           dqkv[:, d:].data_ptr(), 3 * d, sq, dqkv[:, 2 * d:].data_ptr(), 3 * d, sq, K._s())


for _ in range(3):
    bwd()
torch.cuda.synchronize()
lib.mms2ut_diag_attn_phases(None, 0, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
bwd()
e1.record()
torch.cuda.synchronize()
buf = np.zeros(64 * 64, np.uint64)
lib.mms2ut_diag_attn_phases(buf.ctypes.data, buf.size, 0)
st = buf.reshape(64, 64).astype(np.int64)
print(f"B={B} T={T} causal={int(causal)}: kernel {e0.elapsed_time(e1) * 1e3:.1f} us")
names = ["wait b1", "phase1", "phase2", "wait b3", "phase3"]
nch = 0
for c in range(12):
    if (st[:, 1 + 5 * c] == 0).all():
        break
    nch = c + 1
row0 = np.median(st[:, 1] - st[:, 0])
print(f"start -> first chunk: {row0:8.0f} cyc")
for c in range(nch):
    seg = []
    for k in range(5):
        a, b = 1 + 5 * c + k, 2 + 5 * c + k
        ok = (st[:, a] > 0) & (st[:, b] > 0)
        seg.append(np.median(st[ok, b] - st[ok, a]) if ok.any() else float("nan"))
    print(f"chunk {c:2d}: " + "  ".join(f"{n} {v:7.0f}" for n, v in zip(names, seg)))

# forward: per 64-key tile, the wait + stage (top of the tile to after its K/V staging) and the
# compute (S, softmax, PV) cycles, then the epilogue; median over the first 64 blocks
lib.mms2ut_diag_attn_phases(None, 0, 1)
e0.record()
K.call("mms2ut_mha_varlen_fwd", K._attn_args(*args, lens, causal, p, (3, 0), lse, sq=sq, sk=sq, sv=sq, so=T * d),
       K._s())
e1.record()
torch.cuda.synchronize()
lib.mms2ut_diag_attn_phases(buf.ctypes.data, buf.size, 0)
st = buf.reshape(64, 64).astype(np.int64)
print(f"forward kernel {e0.elapsed_time(e1) * 1e3:.1f} us; start -> tile loop {np.median(st[:, 1] - st[:, 0]):7.0f} cyc")
t = 0
while 3 + 2 * t < 40 and (st[:, 3 + 2 * t] > 0).any():
    print(f"tile {t}: stage {np.median(st[:, 3 + 2 * t] - st[:, 2 + 2 * t]):7.0f}  compute "
          f"{np.median((st[:, 4 + 2 * t] if (st[:, 4 + 2 * t] > 0).any() else st[:, 40]) - st[:, 3 + 2 * t]):7.0f}")
    t += 1
print(f"epilogue {np.median(st[:, 41] - st[:, 40]):7.0f} cyc; block total {np.median(st[:, 41] - st[:, 0]):7.0f} cyc")
