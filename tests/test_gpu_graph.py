"""HIP-graph replay of the training step (trainer.Trainer(graph=True)).

1. The device step seed: every dropout kernel family (GEMM epilogues, fused attention, LayerNorm /
   embedding / softmax dropouts) adds the bound device delta to its seed, so a forward with host
   seed s and delta D is bit-identical to one with host seed s + D and nothing bound.
2. Graph mode vs eager: a graph-mode trainer (eager first step per batch, capture, replays) and an
   eager trainer on the same device step-seed schedule agree over several updates, with dropout on
   and modality-dropout branch switches.  Not bit-identical: three reductions use fp32 atomics
   (the loss sum, the attention backward's rowsum(dO*O), the token-embedding gradient), so two
   eager runs already differ in the last bits; the tolerances are that noise (logs 1e-4 relative,
   parameter updates 1e-2 relative), far below what one wrong dropout mask changes (~1e-2 on the
   loss), and the loss scale / step count are exact.
"""
import numpy as np
import pytest
import torch

from conftest import pkg
from oracle import ref_model as R

pytestmark = pytest.mark.gpu


def _cfg(mm, **kw):
    c = R.tiny_config(conv_channels=256)
    c.update(kw)
    return mm.default_cfg(**c)


def _batches(mm, cfg):
    shapes = (([120, 90], [30, 22]), ([100, 77, 60], [25, 20, 15]))
    return [mm.runtime.prepare_batch(mm.data.make_sample(L, T, img_tokens=37, img_dim=768, seed=s), cfg, "cuda")
            for s, (L, T) in enumerate(shapes)]


def test_step_seed_delta_shifts_every_dropout_kernel():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K = mm.kernels
    cfg = _cfg(mm)
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=3)
    model.train()
    batch = _batches(mm, cfg)[1]
    model.np_rng = np.random.RandomState(0)
    D = 0x9E3779B97F4A7C15 * 5 % (1 << 63)
    delta = torch.tensor([D], dtype=torch.int64, device="cuda")
    outs = []
    try:
        for bound in (False, True):
            model.np_rng = np.random.RandomState(0)
            model.drop.reset(7 if bound else 7 + D)
            K.bind_step_seed(delta if bound else None)
            enc, l32, Te, ctx = model.encoder_forward(batch)
            logits, dctx = model.decoder_forward(batch, enc, l32, Te)
            torch.cuda.synchronize()
            # logits' padded vocabulary columns (Vp > V) are never written: compare the V real ones
            outs.append((enc.clone(), logits[..., :cfg["vocab_size"]].clone()))
    finally:
        K.bind_step_seed(None)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    # and the delta does change the masks
    model.np_rng = np.random.RandomState(0)
    model.drop.reset(7)
    enc, *_ = model.encoder_forward(batch)
    assert not torch.equal(enc, outs[0][0])


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.mark.parametrize("mod", [-0.5, 0.5])
def test_graph_trainer_bit_identical_to_eager(mod):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    cfg = _cfg(mm, modality_dropout=mod, audio_dropout=0.5)
    batches = _batches(mm, cfg)
    models = [mm.MMS2UTModel(cfg, device="cuda").init_params(seed=5) for _ in range(2)]
    trs = [mm.trainer.Trainer(models[0], warmup_updates=0, lr=1e-3, graph=True),
           mm.trainer.Trainer(models[1], warmup_updates=0, lr=1e-3, device_seed=True)]
    # step schedule: batch index and (modality, audio) draws -> graph mode captures 0/None, 1/None,
    # replays them, then meets a new branch (audio- or image-dropped) and replays it
    sched = [(0, (0.9, 0.9)), (1, (0.9, 0.9)), (0, (0.9, 0.9)), (1, (0.9, 0.9)),
             (0, (0.1, 0.9)), (1, (0.1, 0.1)), (0, (0.1, 0.9)), (1, (0.1, 0.1)), (0, (0.9, 0.9))]
    p0 = models[1].params.flat.float().clone()
    K = mm.kernels
    try:
        for i, (bi, dr) in enumerate(sched):
            logs = []
            for k, tr in enumerate(trs):
                if k == 0:
                    log = tr.train_step(batches[bi], draws=[dr])
                else:
                    models[1].np_rng = type("S", (), {"v": list(dr), "random": lambda self: self.v.pop(0)})()
                    log = tr.train_step(batches[bi])
                logs.append(log.clone())
            for tr in trs:
                tr.sync()
            torch.cuda.synchronize()
            assert _rel(logs[0], logs[1]) < 1e-4, (i, logs)
            oa, ob = trs[0].opt.ost, trs[1].opt.ost
            for j in (K.OST_LOSS_SCALE, K.OST_STEP, K.OST_OVERFLOW):
                assert oa[j].item() == ob[j].item(), (i, j)
            ua, ub = models[0].params.flat.float() - p0, models[1].params.flat.float() - p0
            if ub.norm() > 0:
                assert _rel(ua, ub) < 1e-2, (i, _rel(ua, ub))
            assert _rel(trs[0].opt.master - p0, trs[1].opt.master - p0) < 1e-2, i
        n = len(trs[0].graphs)
        assert n == (2 if mod < 0 else 4), n
    finally:
        mm.kernels.bind_step_seed(None)


def test_stream_workspace_retired_in_graph_mode():
    """A regrown per-stream split-K workspace is retired (kept alive) in graph mode: a graph
    captured with the smaller buffer keeps writing into it on every replay (kernels.stream_workspace)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    K = pkg().kernels
    side = K._Side
    saved = (side.retain, list(side.retired))
    try:
        side.retain = True
        small = K.stream_workspace(1 << 20, "cuda")
        big = K.stream_workspace(4 << 20, "cuda")
        assert big.data_ptr() != small.data_ptr() and big.numel() >= 4 << 20
        assert any(t.data_ptr() == small.data_ptr() for t in side.retired)
        assert K.stream_workspace(2 << 20, "cuda").data_ptr() == big.data_ptr()   # no regrowth below the size
    finally:
        side.retain, side.retired[:] = saved[0], saved[1]
