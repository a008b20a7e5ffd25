"""Is the host ahead of the GPU?  For each step record (host time, GPU event) at step start, after the
forward issue and after the backward issue; print how far the GPU trails the host at each point.
A GPU that completes a point right when the host issued it (lag ~ 0) is starved by host issue.

usage: python scripts/host_lag.py [steps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
mm = bench.mm
device = torch.device("cuda", 0)
cfg = mm.default_cfg()
model = mm.MMS2UTModel(cfg, device=device).init_params(seed=1)
tr = bench.trainer_mod.Trainer(model, lr=5e-4, world_size=1)
fe = bench.frontend_mod.FbankFrontend(device)
batches = bench.make_batches(cfg, 0, 8, 40000, device, fe)
marks = []
orig_ce = bench.runtime.label_smoothed_ce


def mark(tag):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    marks.append((tag, time.perf_counter(), e))


def ce(*a, **k):
    mark("fwd_issued")
    return orig_ce(*a, **k)


bench.runtime.label_smoothed_ce = ce
orig_step = tr.opt.step


def opt_step(*a, **k):
    mark("bwd_issued")
    return orig_step(*a, **k)


tr.opt.step = opt_step


def step(i):
    wb, batch = batches[i % len(batches)][:2]
    mark("start")
    batch.src = fe(wb)
    tr.train_step(batch)


for i in range(3):
    step(i)
torch.cuda.synchronize()
marks.clear()
for i in range(steps):
    step(3 + i)
mark("end")
torch.cuda.synchronize()
t0h, e0 = marks[0][1], marks[0][2]
print(f"{'mark':12s} {'host ms':>9s} {'gpu ms':>9s} {'gpu-host':>9s}")
for tag, th, e in marks:
    tg = e0.elapsed_time(e)
    print(f"{tag:12s} {1e3 * (th - t0h):9.2f} {tg:9.2f} {tg - 1e3 * (th - t0h):9.2f}")
