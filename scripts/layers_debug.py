"""Debug: one-call layers vs per-launch layers, stage by stage (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import pkg  # noqa: E402

mm = pkg()
K = mm.kernels
cfg = mm.default_cfg(encoder_layers=2, decoder_layers=2)
lengths, tlens = [700, 640, 560, 500], [211, 193, 169, 151]
model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=8)
sample = mm.data.make_sample(lengths, tlens, img_tokens=577, img_dim=768, seed=5)
batch = mm.runtime.prepare_batch(sample, cfg, "cuda")
M = type(model)


class _Draws:
    def random(self):
        return 0.99


def use(ref):
    for n in ("enc_layer_fwd", "enc_layer_bwd", "dec_layer_fwd", "dec_layer_bwd"):
        model.__dict__.pop(n, None)
        if ref:
            setattr(model, n, getattr(M, n + "_ref").__get__(model))


def run(ref, tag):
    use(ref)
    model.drop.reset(4321)
    model.np_rng = _Draws()
    model.params.grad.zero_()
    p0 = model.params.flat.float().sum().item()
    logits = mm.runtime.model_logits(model, batch)
    out = logits.clone()
    torch.cuda.synchronize()
    loss, _ = mm.runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"], 0.2, 1)
    loss.backward(torch.tensor(16.0, device="cuda"))
    torch.cuda.synchronize()
    p1 = model.params.flat.float().sum().item()
    print(tag, "params sum before/after", p0, p1, "loss", float(loss), "logits absmax", float(out.abs().max()),
          "TW active", K.TransposedWeights.active, flush=True)
    return out, model.params.grad.clone()


a = run(False, "new1")
b = run(True, "ref1")
c = run(False, "new2")
d = run(True, "ref2")
for (x, gx), (y, gy), name in ((a, c, "new1-new2"), (b, d, "ref1-ref2"), (a, b, "new1-ref1"), (c, d, "new2-ref2")):
    dl = (x.float() - y.float()).abs()
    bad = (dl > 0).nonzero()
    print(name, "logits equal", torch.equal(x, y), "maxdiff", float(dl.max()), "nbad", bad.shape[0],
          "first bad", bad[:5].tolist(), "grads equal", torch.equal(gx, gy), flush=True)
    if bad.shape[0]:
        cols = bad[:, 1]
        rows = bad[:, 0]
        print("   bad cols range", int(cols.min()), int(cols.max()), "rows range", int(rows.min()), int(rows.max()),
              "shape", tuple(x.shape))

# per-layer forward on identical input
use(False)
model.drop.reset(99)
x = torch.randn(4 * 700, cfg["encoder_embed_dim"], device="cuda").half()
lens = torch.tensor(lengths, dtype=torch.int32, device="cuda")
y_new, cn = model.enc_layer_fwd(0, x, 4, 700, lens)
model.drop.reset(99)
y_ref, cr = M.enc_layer_fwd_ref(model, 0, x, 4, 700, lens)
torch.cuda.synchronize()
print("enc layer fwd equal", torch.equal(y_new, y_ref), float((y_new.float() - y_ref.float()).abs().max()))
for k in ("f1",):
    print(" ", k, torch.equal(cn[k], cr[k]))
