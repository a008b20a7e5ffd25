"""Per-tensor bit checksums of one seeded base-model forward + backward (library under test:
MMS2UT_LIB): the loss, the logits, every encoder / decoder layer's input gradient and every
parameter gradient slice.  Two libraries that should be bit-identical print identical JSON; where
they are not, the first differing tensors name the kernel family.
usage: python scripts/step_grads.py OUT.json"""
import hashlib
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
mm = importlib.import_module("multimodal-s2ut_amd")
from oracle import ref_model as R  # noqa: E402  (parameter init only: the seeded base weights)


def h(t):
    return hashlib.sha1(t.detach().contiguous().cpu().view(torch.uint8).numpy().tobytes()).hexdigest()[:12]


cfg = R.base_config()
P = {k: v.half().float() for k, v in R.init_params(cfg, seed=7, include_unused=False).items()}
model = mm.MMS2UTModel(mm.default_cfg(**cfg), device="cuda")
model.params.load_state_dict(P, strict=True)
lengths = [1000, 900, 800, 700, 640, 560, 520, 500]
sample = mm.data.make_sample(lengths, [round(0.3 * L) + 1 for L in lengths], img_tokens=577,
                             img_dim=cfg["image_feat_dim"], seed=3)
batch = mm.runtime.prepare_batch(sample, model.cfg)
out = {}
eb, db = model.enc_layer_bwd, model.dec_layer_bwd


def enc_bwd(l, *a, **k):
    r = eb(l, *a, **k)
    out[f"enc_dx{l}"] = h(r[0])
    return r


def dec_bwd(l, *a, **k):
    r = db(l, *a, **k)
    out[f"dec_dx{l}"] = h(r[0])
    return r


model.enc_layer_bwd, model.dec_layer_bwd = enc_bwd, dec_bwd
model.drop.reset(1234)
model.params.grad.zero_()
logits = mm.runtime.model_logits(model, batch)
loss, nll = mm.runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"], cfg["label_smoothing"], 1)
out["logits"] = h(logits)
out["loss"] = float(loss)
loss.backward(torch.tensor(16.0, device="cuda"))
torch.cuda.synchronize()
for name, g in model.params.g.items():
    out["grad:" + name] = h(g)
out["grad_all"] = h(model.params.grad)
json.dump(out, open(sys.argv[1], "w"), indent=0)
print(json.dumps(out)[:400])
