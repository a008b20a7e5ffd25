"""Isolated timing of the fused attention kernels on the step's shapes (packed QKV layout as in
the encoder: q/k/v are column slices of one [B*T, 3d] buffer).  Usage: python scripts/attn_bench.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels


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


def case(B, T, H=8, d=768, p=0.1, causal=False):
    hd = d // H
    dev = "cuda"
    qkv = torch.randn(B * T, 3 * d, device=dev).half()
    O = torch.empty(B * T, d, dtype=torch.float16, device=dev)
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    args = (qkv, qkv[:, d:], qkv[:, 2 * d:], O, 3 * d, 3 * d, 3 * d, d, B, H, T, T, hd, hd ** -0.5)
    kw = dict(key_len=lens, causal=causal, p=p, drop=(3, 0))
    sq = T * 3 * d
    fwd = lambda: K.call("mms2ut_mha_varlen_fwd", K._attn_args(*args, kw["key_len"], causal, p, kw["drop"],  # noqa: E731
                                                               lse, sq=sq, sk=sq, sv=sq, so=T * d), K._s())
    lse = torch.empty(B * H * T, dtype=torch.float32, device=dev)
    tf = timeit(fwd)
    dO = torch.randn(B * T, d, device=dev).half()
    dqkv = torch.empty_like(qkv)
    Dd = torch.empty(B * H * T, dtype=torch.float32, device=dev)

    def bwd():
        a = K._attn_args(*args, kw["key_len"], causal, p, kw["drop"], lse, sq=sq, sk=sq, sv=sq, so=T * d)
        K.call("mms2ut_mha_varlen_bwd", a, dO.data_ptr(), d, T * d, Dd.data_ptr(), dqkv.data_ptr(), 3 * d, sq,
               dqkv[:, d:].data_ptr(), 3 * d, sq, dqkv[:, 2 * d:].data_ptr(), 3 * d, sq, K._s())
    tb = timeit(bwd)
    fl = 4.0 * B * H * T * T * hd * (0.5 if causal else 1.0)
    byts = 4 * B * T * d * 2
    print(f"B={B:3d} T={T:4d} p={p} causal={int(causal)}  fwd {tf:7.1f} us {fl / tf / 1e6:6.1f} TF "
          f"{byts / tf / 1e3:6.0f} GB/s   bwd {tb:7.1f} us {2.5 * fl / tb / 1e6:6.1f} TF", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # one case: B T p [causal]
        case(int(sys.argv[1]), int(sys.argv[2]), p=float(sys.argv[3]),
             causal=len(sys.argv) > 4 and sys.argv[4] == "1")
        sys.exit(0)
    case(95, 106)
    case(95, 106, p=0.0)
    case(95, 128, p=0.0)
    case(40, 250)
    case(95, 128, causal=True)
    case(32, 301, causal=True)
    case(85, 142, causal=True)
    case(68, 177, causal=True)
    case(68, 250, causal=True)
