"""Cost of a main->side stream fork on the main stream: a chain of small kernels on the current
stream, with (a) nothing between them, (b) mms2ut_stream_wait(side, main) after each (event record
+ wait), (c) hipStreamWriteValue32 on main + hipStreamWaitValue32 on side."""
import ctypes
import importlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels
hip = ctypes.CDLL("libamdhip64.so")


def run(mode, n=200):
    x = torch.randn(1 << 20, device="cuda").half()
    y = torch.empty_like(x)
    side = torch.cuda.Stream(priority=100)
    main = torch.cuda.current_stream()
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        K.call("mms2ut_add_f16", x.data_ptr(), x.data_ptr(), y.data_ptr(), x.numel(), K._s())
        if mode == "event":
            K.call("mms2ut_stream_wait", side.cuda_stream, main.cuda_stream)
        elif mode == "value":
            hip.hipStreamWriteValue32(ctypes.c_void_p(main.cuda_stream), ctypes.c_void_p(flag.data_ptr()),
                                      ctypes.c_uint32(i + 1), ctypes.c_uint32(0))
            hip.hipStreamWaitValue32(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(flag.data_ptr()),
                                     ctypes.c_uint32(i + 1), ctypes.c_uint32(0), ctypes.c_uint32(0xffffffff))
        elif mode == "torch":
            side.wait_stream(main)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for mode in ["none", "event", "value", "torch", "none", "event"]:
    run(mode, 20)
    print(f"{mode:6s} {run(mode):7.2f} us per kernel", flush=True)
