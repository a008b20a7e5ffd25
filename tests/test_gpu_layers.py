"""GPU: the one-call transformer layers (include/mms2ut.h mms2ut_layer_fwd / mms2ut_layer_bwd,
csrc/layers.hip), the one-call Conv1d subsampler (mms2ut_conv1d_glu_fwd / _bwd) and the one-call
fusion tail (mms2ut_gated_fusion_fwd / _bwd) match the per-launch path they replace
(model.enc_layer_*_ref / dec_layer_*_ref / subsample_*_ref / fusion_*_ref, the
kernel-by-kernel sequence the oracle parity tests pinned): logits, every
parameter gradient and the encoder-output gradient, dropout on at every site, on the base dims
and on a short batch whose GEMMs take the split-K fixup path.  Also checks the layers with the
weight-gradient side stream folded into the main stream (the bench's roofline pass)."""
import re

import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg()


class _Draws:
    def random(self):
        return 0.99


def _step(mm, model, batch, cfg, ref):
    M = type(model)
    if ref:
        model.enc_layer_fwd = M.enc_layer_fwd_ref.__get__(model)
        model.enc_layer_bwd = M.enc_layer_bwd_ref.__get__(model)
        model.dec_layer_fwd = M.dec_layer_fwd_ref.__get__(model)
        model.dec_layer_bwd = M.dec_layer_bwd_ref.__get__(model)
        model.subsample_fwd = M.subsample_fwd_ref.__get__(model)
        model.subsample_bwd = M.subsample_bwd_ref.__get__(model)
        model.fusion_fwd = M.fusion_fwd_ref.__get__(model)
        model.fusion_bwd = M.fusion_bwd_ref.__get__(model)
    else:
        for n in ("enc_layer_fwd", "enc_layer_bwd", "dec_layer_fwd", "dec_layer_bwd", "subsample_fwd", "subsample_bwd",
                  "fusion_fwd", "fusion_bwd"):
            model.__dict__.pop(n, None)
    model.drop.reset(4321)
    model.np_rng = _Draws()
    model.params.grad.zero_()
    stash = {}
    eb = model.encoder_backward

    def enc_bwd(ctx, denc, dstates=None):
        stash["denc"] = denc.clone()
        return eb(ctx, denc, dstates)
    model.encoder_backward = enc_bwd
    try:
        logits = mm.runtime.model_logits(model, batch)
        out = logits[:, :cfg["vocab_size"]].clone()     # columns past V: GEMM row padding, never written
        loss, _ = mm.runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"], 0.2, 1)
        loss.backward(torch.tensor(16.0, device="cuda"))
        torch.cuda.synchronize()
    finally:
        model.__dict__.pop("encoder_backward", None)
    return out, model.params.grad.clone(), stash["denc"], float(loss)


@pytest.mark.parametrize("case", ["base", "short_fixup", "side_folded", "selective_detr", "no_prenorm"])
def test_layer_calls_bit_identical_to_per_launch(mm, case):
    K = mm.kernels
    img_tokens, img_dim = 577, 768
    if case == "short_fixup":
        cfg = mm.default_cfg(encoder_layers=2, decoder_layers=2)
        lengths, tlens = [90, 70], [25, 20]            # M = B*T of a few hundred rows: fixup splits
    elif case == "selective_detr":
        # selective attention (no bias_kv), DETR features (Di = 256 != d: separate k|v weights),
        # no gate (plain residual), SA_image_dropout 0.5 through the fused image LayerNorm
        cfg = mm.default_cfg(encoder_layers=1, decoder_layers=1, multimodal_attention_type="selective_attention",
                             image_feat_dim=256, use_selective_gate=False, SA_image_dropout=0.5)
        lengths, tlens = [600, 500, 420], [181, 151, 127]
        img_tokens, img_dim = 100, 256
    elif case == "no_prenorm":
        # multimodal attention without the image LayerNorm: image dropout + bias_kv key layout copy
        cfg = mm.default_cfg(encoder_layers=1, decoder_layers=1, image_pre_norm=False, SA_image_dropout=0.3,
                             SA_text_dropout=0.2)
        lengths, tlens = [500, 430], [151, 130]
    else:
        cfg = mm.default_cfg(encoder_layers=2, decoder_layers=2)
        lengths, tlens = [700, 640, 560, 500], [211, 193, 169, 151]
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=8)
    sample = mm.data.make_sample(lengths, tlens, img_tokens=img_tokens, img_dim=img_dim, seed=5)
    batch = mm.runtime.prepare_batch(sample, cfg, "cuda")
    side = K._Side.enabled
    if case == "side_folded":
        K._Side.enabled = False
    try:
        lg_n, g_n, de_n, l_n = _step(mm, model, batch, cfg, ref=False)
        lg_r, g_r, de_r, l_r = _step(mm, model, batch, cfg, ref=True)
    finally:
        K._Side.enabled = side
    assert torch.equal(lg_n, lg_r)
    assert l_n == l_r                       # the loss reduction is fixed-order too
    assert torch.equal(de_n, de_r)
    # weight gradients: the one-call layers issue each layer's projections as one grouped, unsplit
    # launch (fp32 accumulation over all rows), the per-launch path splits K into fp32 slabs — the
    # same products in another summation order; everything else is bit-identical
    lw = [n for n in model.params.offsets if re.search(r"layers\.\d+\.(self_attn|encoder_attn)\.(q|k|v|out)_proj\.|"
                                                       r"layers\.\d+\.fc[12]\.", n) and "encoder_attn.k_proj" not in n
          and "encoder_attn.v_proj" not in n]
    assert lw
    for n, (o, _, k) in model.params.offsets.items():
        a, b = g_n[o:o + k].float(), g_r[o:o + k].float()
        if n in lw:
            assert float((a - b).norm()) <= 2e-3 * float(b.norm()) + 1e-6, n
        else:
            assert torch.equal(g_n[o:o + k], g_r[o:o + k]), n
    assert float(g_n.float().norm()) > 0
