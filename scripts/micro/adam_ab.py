"""Isolated Adam (fp16 params, fp32 master / moments) over one optimizer chunk of the step's size,
timed with HIP events over 50 launches (the round-5 A/B built its variants behind an MMS_ADAM_V
switch, since removed: profiles/round5_adam_ab.txt).  Prints the mean launch time, the HBM rate at 28 B per parameter and a checksum of the
updated buffers (variants must agree bit for bit)."""
import hashlib
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
K = importlib.import_module("multimodal-s2ut_amd.kernels")

n = int(os.environ.get("ADAM_N", 6_840_000))
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
param = torch.empty(n, dtype=torch.float16, device=dev)
grad = (torch.randn(n, generator=g, device=dev) * 1e-2).half()
master = torch.randn(n, generator=g, device=dev)
m = torch.randn(n, generator=g, device=dev) * 1e-3
v = torch.rand(n, generator=g, device=dev) * 1e-5
ost = torch.zeros(16, dtype=torch.float32, device=dev)
ost[0] = 1.0       # MULT
ost[4] = 1e-4      # STEP_SIZE
ost[9] = 1.0       # CLIP_COEF
ost[11] = 5e-4     # LR
K.adam(param, grad, master, m, v, ost, 0.9, 0.98, 1e-8, 0.0)
torch.cuda.synchronize()
h = hashlib.sha1()
for t in (param, master, m, v):
    h.update(t.cpu().numpy().tobytes())
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(5):
    K.adam(param, grad, master, m, v, ost, 0.9, 0.98, 1e-8, 0.0)
a.record()
R = 50
for _ in range(R):
    K.adam(param, grad, master, m, v, ost, 0.9, 0.98, 1e-8, 0.0)
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) * 1e3 / R
print(f"adam V={os.environ.get('MMS_ADAM_V', '0')} n={n}: {us:.2f} us/launch, {28 * n / us / 1e6:.3f} TB/s, "
      f"sha1(first update) {h.hexdigest()[:16]}", flush=True)
