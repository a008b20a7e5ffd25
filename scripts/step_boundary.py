"""Step boundary of the unprofiled bench loop: when, relative to the deferred Adam chunks on the side
stream, does the next step's front end (and its first encoder layer) run?  Timing events on
the three streams: main-stream end of step k (after optim_prepare), side-stream end of step k's
Adam chunks, current-stream end of step k + 1's fbank + CMVN, main-stream end of its first
forward GEMM group.  (A rocprofv3 kernel trace throttles the host to ~0.5 ms ahead of the GPU, so
its step boundary is not the bench's.)   usage: python scripts/step_boundary.py [steps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

K = bench.kernels
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
device = torch.device("cuda", 0)
torch.cuda.set_device(device)
cfg = bench.mm.default_cfg()
model = bench.mm.MMS2UTModel(cfg, device=device).init_params(seed=1)
tr = bench.trainer_mod.Trainer(model, lr=5e-4, world_size=1)
fe = bench.frontend_mod.FbankFrontend(device)
batches = bench.make_batches(cfg, 0, 8, 40000, device, fe)


def ev(stream):
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


rec = []


def step(i, log):
    wb, batch = batches[i % len(batches)][:2]
    cur = torch.cuda.current_stream()

    def frontend():
        batch.src = fe(wb)
        if log:
            rec[-1]["fbank_done"] = ev(cur)
    if log:
        rec.append({"start": ev(cur)})
    tr.train_step(batch, prologue=frontend)
    if log:
        rec[-1]["main_done"] = ev(tr.stream)
        rec[-1]["side_done"] = ev(K.side_stream(device))


for i in range(4):
    step(i, False)
torch.cuda.synchronize()
for i in range(steps):
    step(4 + i, True)
torch.cuda.synchronize()
t0 = rec[0]["start"]
print("step  start  fbank_done  main_done  side_done   (ms from the first logged start)")
for k, r in enumerate(rec):
    print(f"{k:4d} " + "  ".join(f"{t0.elapsed_time(r[n]):9.3f}" for n in ("start", "fbank_done", "main_done", "side_done")))
for k in range(1, len(rec)):
    a = rec[k - 1]
    b = rec[k]
    print(f"step {k}: fbank_done - prev main_done {a['main_done'].elapsed_time(b['fbank_done']) * 1e3:8.1f} us;"
          f" fbank_done - prev side_done {a['side_done'].elapsed_time(b['fbank_done']) * 1e3:8.1f} us;"
          f" step {a['main_done'].elapsed_time(b['main_done']):7.3f} ms")
