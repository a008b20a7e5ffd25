"""The hand-written backward defines every parameter gradient outright (round 5: the trainer no
longer clears the 301 MB flat gradient buffer each step).

For every model variant and modality-dropout branch the step can take, one training forward +
backward runs twice on the same inputs, dropout seed and forced draws: once with the gradient
buffer cleared, once with it poisoned (every element NaN).  The two gradient buffers must be
bit-identical and finite — a parameter whose gradient some branch neither writes nor zeroes
(model._zero_grads) would keep the poison.  Reference: fairseq zeroes .grad before every
backward (Trainer.train_step -> optimizer.zero_grad), which is what the poisoned run must match.
"""
import pytest
import torch

from conftest import pkg
from oracle import ref_model as R
from parity_util import MODALITY_DRAWS, _Draws

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg()


SMALL = dict(conv_channels=256, encoder_embed_dim=128, encoder_ffn_embed_dim=512, encoder_attention_heads=2,
             decoder_embed_dim=128, decoder_ffn_embed_dim=512, decoder_attention_heads=2)

VARIANTS = {
    "gate_vit": dict(image_feat_dim=128),
    "selective": dict(image_feat_dim=128, multimodal_attention_type="selective_attention"),
    "detr_qkv": dict(image_feat_dim=64),                       # Di != d: separate q/k/v projections
    "no_gate": dict(image_feat_dim=128, use_selective_gate=False),
    "qformer": dict(image_feat_dim=128, multimodal_extractor_type="q_former", num_queries=6,
                    num_query_layers=2, num_multimodal_layers=1),
    "external1": dict(image_feat_dim=128, multimodal_attention_type="external_multimodal_transformer",
                      external_multimodal_transformer_layers=1),
    "external2": dict(image_feat_dim=128, multimodal_attention_type="external_multimodal_transformer",
                      external_multimodal_transformer_layers=2),
    "audio_only": dict(fusion=False),
}


def _step_grads(mm, model, batch, cfg, modality, poison):
    model.drop.reset(1234)
    model.np_rng = _Draws(MODALITY_DRAWS[modality])
    model.params.await_all()
    if poison:
        model.params.grad.fill_(float("nan"))
    else:
        model.params.grad.zero_()
    logits, aux = mm.runtime.model_outputs(model, batch)
    loss, _ = mm.runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"], cfg["label_smoothing"], 1)
    (loss + aux if aux is not None else loss).backward(torch.tensor(16.0, device="cuda"))
    torch.cuda.synchronize()
    return model.params.grad.clone()


def _check(mm, cfg, modality, with_images=True):
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=7)
    sample = mm.data.make_sample([150, 121, 97], [41, 30, 22], img_tokens=37, img_dim=cfg["image_feat_dim"],
                                 with_images=with_images, img_mask=with_images, seed=3)
    batch = mm.runtime.prepare_batch(sample, cfg, "cuda")
    ref = _step_grads(mm, model, batch, cfg, modality, poison=False)
    got = _step_grads(mm, model, batch, cfg, modality, poison=True)
    bad = [n for n, (off, _, k) in model.params.offsets.items() if not torch.isfinite(got[off:off + k]).all()]
    assert not bad, f"gradients left unwritten: {bad[:8]}"
    diff = _differing(model, ref, got)
    assert not diff, diff[:8]


def _differing(model, a, b):
    """Parameters whose gradient bits differ between two runs."""
    a16, b16 = a.view(torch.int16), b.view(torch.int16)
    return [n for n, (off, _, k) in model.params.offsets.items() if not torch.equal(a16[off:off + k], b16[off:off + k])]


@pytest.mark.parametrize("modality", [None, "audio", "image"])
@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_backward_writes_every_gradient(mm, variant, modality):
    if variant == "audio_only" and modality is not None:
        pytest.skip("no fusion: no modality dropout")
    over = dict(SMALL, **VARIANTS[variant])
    if modality is not None:
        over.update(modality_dropout=1.0, audio_dropout=1.0 if modality == "audio" else 0.0)
    cfg = mm.default_cfg(**R.tiny_config(**over))
    _check(mm, cfg, modality)


def test_backward_writes_every_gradient_without_images(mm):
    """A fusion model fed a batch without image features: the fusion tail does not run."""
    cfg = mm.default_cfg(**R.tiny_config(**dict(SMALL, image_feat_dim=128)))
    _check(mm, cfg, None, with_images=False)


def test_backward_writes_every_gradient_multitask(mm):
    """Auxiliary decoder / CTC heads on encoder and decoder states (multitask.py)."""
    from test_gpu_multitask import _mt_sample, _tasks
    cfg = mm.default_cfg(**R.tiny_config(conv_channels=256))
    letters, tasks = _tasks(mm, cfg)
    cfg["multitask"] = tasks
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=9)
    sample = mm.data.make_sample([160, 131, 97], [41, 30, 22], img_tokens=37, img_dim=768, seed=2)
    sample["multitask"] = _mt_sample(mm, tasks, letters, sample, seed=3)
    batch = mm.runtime.prepare_batch(sample, cfg, "cuda")
    ref = _step_grads(mm, model, batch, cfg, None, poison=False)
    got = _step_grads(mm, model, batch, cfg, None, poison=True)
    bad = [n for n, (off, _, k) in model.params.offsets.items() if not torch.isfinite(got[off:off + k]).all()]
    assert not bad, f"gradients left unwritten: {bad[:8]}"
    # the auxiliary heads' token-embedding scatter sums duplicate tokens of the small letter
    # vocabulary in arrival order (fp32), so two runs agree to rounding, not bit for bit
    for n in _differing(model, ref, got):
        off, _, k = model.params.offsets[n]
        a, b = ref[off:off + k].float(), got[off:off + k].float()
        assert (a - b).norm() <= 1e-3 * a.norm() + 1e-6, n
