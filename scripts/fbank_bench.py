"""Isolated timing of the fbank kernel on a bench-sized batch (40 utterances of clip(N(400,120),
150, 1000) x 160 samples: ~16k-30k frames), HIP events over 20 calls; prints us, frames and the
achieved HBM rate (4 B per input sample read + 4 * nbins B per frame written, the §8d count)."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
fe = mm.frontend.FbankFrontend("cuda")
rng = np.random.default_rng(0)
for nutt in (40, 80):
    T = np.clip(rng.normal(400, 120, nutt), 150, 1000).astype(int) * 4   # fbank frames = 4 x encoder frames
    waves = [(rng.standard_normal(160 * t + 240) * 3000).astype(np.float32) for t in T]
    wb = fe.upload(waves)
    for _ in range(3):
        fe.features_f32(wb)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        fe.features_f32(wb)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    frames = int(wb["frame_off"][-1])
    samples = sum(len(w) for w in waves)
    by = 4.0 * samples + 4.0 * 80 * frames
    print(f"fbank B={nutt} frames={frames}: {us:.1f} us  {by / us / 1e3:.0f} GB/s  ({by / 1e6:.1f} MB)", flush=True)
