"""GPU: the trainer's deferred, chunked Adam (optimizer update on the side stream, awaited group
by group by the next forward) gives bit-identical parameters and optimizer state to the
in-order update over several steps; the forward-consumption groups tile the flat buffer."""

import pytest
import torch

from conftest import pkg
from oracle import ref_model as R

pytestmark = pytest.mark.gpu


def _run(defer, steps=3):
    mm = pkg()
    cfg = mm.default_cfg(**R.no_dropout(R.tiny_config(conv_channels=256)))
    model = mm.MMS2UTModel(cfg, device="cuda:0").init_params(seed=4)
    tr = mm.trainer.Trainer(model, lr=1e-3, warmup_updates=2, world_size=1)
    tr.opt.defer = defer
    sample = mm.data.make_sample([61, 47, 30], [14, 11, 9], img_tokens=17, img_dim=cfg["image_feat_dim"], seed=2)
    batch = mm.runtime.prepare_batch(sample, model.cfg, "cuda:0")
    for _ in range(steps):
        tr.train_step(batch)
    st = tr.opt.stats()
    torch.cuda.synchronize()
    return model.params.flat.clone(), tr.opt.master.clone(), tr.opt.exp_avg_sq.clone(), st


def test_deferred_adam_bit_identical():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p0, m0, v0, s0 = _run(False)
    p1, m1, v1, s1 = _run(True)
    assert s0 == s1
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1)
