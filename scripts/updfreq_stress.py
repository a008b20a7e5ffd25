"""Repeatability of the single-process --update-freq 2 gradient (the reference side of
tests/test_gpu_dp.py::test_dp_gradient_equals_accumulated_union): a fresh trainer per round on the
DP test's tiny model and batches, the first step's final fp16 gradient hashed; every round must give
the same bits.  usage: python scripts/updfreq_stress.py [rounds]"""
import hashlib
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
mm = importlib.import_module("multimodal-s2ut_amd")
from dp_common import batches, model_cfg  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = model_cfg(mm)
bs = batches(mm, cfg)
seen = {}
for r in range(rounds):
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=5)
    tr = mm.trainer.Trainer(model, lr=1e-3, world_size=1, init_scale=8.0, warmup_updates=0, update_freq=2)
    taps = []
    tr.grad_tap = lambda g: taps.append(g.clone()) if not taps else None
    tr.train_step(bs)
    torch.cuda.synchronize()
    h = hashlib.sha1(taps[0].cpu().view(torch.uint8).numpy().tobytes()).hexdigest()[:12]
    seen.setdefault(h, []).append(r)
    print(f"round {r}: {h}", flush=True)
    tr.sync()
print("distinct gradients:", len(seen), {k: len(v) for k, v in seen.items()})
sys.exit(0 if len(seen) == 1 else 1)
