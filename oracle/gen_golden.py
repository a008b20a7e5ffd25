"""Golden-vector generator for the gated image-fusion block (TEST INFRASTRUCTURE ONLY).

Runs the reference's OWN fusion code (``mm_s2ut/models/fuse.py:35-167`` and
``MM_S2STransformerEncoder.fuse_img_feat`` at ``mm_s2ut/models/mm_s2s_transformer.py:594-622``)
under an in-memory import shim that serves placeholder modules for the absent third-party
packages ``fairseq`` / ``timm`` / ``omegaconf``.  Only fairseq's base
classes are stubbed; the fusion arithmetic itself is executed verbatim from /root/reference.

Output: ``tests/golden/fusion_*.npz`` — inputs, every parameter, outputs and gradients, in
float64.  This script contains no reference source and never runs on the GPU box: it needs
``/root/reference`` and skips itself when that is absent.  Regenerate with

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py
"""
import importlib.abc
import importlib.machinery
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def _install_shim():
    sys.path.insert(0, REF)

    class Anything(nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

        def __call__(self, *a, **k):
            return a[0] if len(a) == 1 and isinstance(a[0], type) else self

    class AutoMod(types.ModuleType):
        def __getattr__(self, name):
            if name.startswith("__"):
                raise AttributeError(name)
            if name == "Linear":
                def Linear(i, o, bias=True):
                    m = nn.Linear(i, o, bias)
                    nn.init.xavier_uniform_(m.weight)
                    if bias:
                        nn.init.constant_(m.bias, 0.0)
                    return m
                return Linear
            if name == "with_incremental_state":
                return lambda c: c
            if name in ("register_model", "register_model_architecture",
                        "register_task", "register_criterion"):
                return lambda *a, **k: (lambda c: c)
            return type(name, (Anything,), {})

    class Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
        def find_spec(self, name, path, target=None):
            if name.split(".")[0] in ("fairseq", "timm", "omegaconf"):
                return importlib.machinery.ModuleSpec(name, self, is_package=True)
            return None

        def create_module(self, spec):
            m = AutoMod(spec.name)
            m.__path__ = []
            return m

        def exec_module(self, m):
            pass

    sys.meta_path.insert(0, Finder())


class MaskDropout(nn.Module):
    """Dropout with an injected keep-mask (so a GPU kernel can replay the exact mask)."""

    def __init__(self, p, mask):
        super().__init__()
        self.p = p
        self.mask = mask

    def forward(self, x):
        if self.p <= 0:
            return x
        return x * self.mask.to(x.dtype) / (1.0 - self.p)


def _make_case(M, F, name, *, att, gate, d, Di, B, Te, Ti, text_pad, img_pad,
               p_img=0.0, p_txt=0.0, p_attn=0.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    h = nn.Module()
    h.image_pre_norm_module = nn.LayerNorm([Di], 1e-5, True)
    with torch.no_grad():
        h.image_pre_norm_module.weight.copy_(1.0 + 0.1 * torch.randn(Di, generator=g))
        h.image_pre_norm_module.bias.copy_(0.1 * torch.randn(Di, generator=g))
    img_keep = (torch.rand(Ti, B, Di, generator=g) >= p_img)
    txt_keep = (torch.rand(Te, B, d, generator=g) >= p_txt)
    attn_keep = (torch.rand(B, Te, Ti, generator=g) >= p_attn)
    h.image_dropout_module = MaskDropout(p_img, img_keep)
    h.text_dropout_module = MaskDropout(p_txt, txt_keep)
    h.gate_denses = nn.ModuleList([M.Linear(2 * d, d)])
    with torch.no_grad():
        h.gate_denses[0].bias.copy_(0.1 * torch.randn(d, generator=g))
    h.use_selective_gate = gate
    h.is_merge_text_img = False
    h.multimodal_attention_type = att
    if att == "selective_attention":
        sa = F.SelectiveAttention(qdim=d, kdim=Di, vdim=Di, attn_dim=d, intermediate_dim=d,
                                  output_dim=d, num_heads=1, attn_drop=p_attn)
        with torch.no_grad():
            for lin in (sa.q_proj, sa.k_proj, sa.v_proj, sa.proj):
                lin.bias.copy_(0.1 * torch.randn(lin.bias.shape, generator=g))
        sa.attn_drop = MaskDropout(p_attn, attn_keep)
        h.selective_attns = nn.ModuleList([sa])
    else:
        assert p_attn == 0.0, "nn.MultiheadAttention dropout cannot be replayed"
        ma = F.MultimodalAttention(embed_dim=d, kdim=Di, vdim=Di, num_heads=1,
                                   dropout=p_attn, add_bias_kv=True)
        with torch.no_grad():
            ma.in_proj_bias.copy_(0.1 * torch.randn(3 * d, generator=g))
            ma.out_proj.bias.copy_(0.1 * torch.randn(d, generator=g))
        h.multimodal_attns = nn.ModuleList([ma])
    h = h.double()
    h.train()
    for mod in (h.image_dropout_module, h.text_dropout_module):
        mod.mask = mod.mask
    text = torch.randn(Te, B, d, generator=g, dtype=torch.float64).requires_grad_(True)
    img = torch.randn(Ti, B, Di, generator=g, dtype=torch.float64)
    text_len = torch.full((B,), Te, dtype=torch.long)
    if text_pad:
        text_len = torch.randint(max(1, Te // 2), Te + 1, (B,), generator=g)
        text_len[0] = Te
    text_mask = torch.arange(Te)[None, :] >= text_len[:, None]
    img_mask = None
    if img_pad:
        img_len = torch.randint(max(1, Ti // 2), Ti + 1, (B,), generator=g)
        img_len[0] = Ti
        img_mask = torch.arange(Ti)[None, :] >= img_len[:, None]
    res, mask_out = M.MM_S2STransformerEncoder.fuse_img_feat(h, text, 0, img, img_mask, text_mask)
    gout = torch.randn(res.shape, generator=g, dtype=torch.float64)
    (res * gout).sum().backward()
    out = dict(
        att=np.array(att), gate=np.array(gate), d=np.array(d), Di=np.array(Di),
        p_img=np.array(p_img), p_txt=np.array(p_txt), p_attn=np.array(p_attn),
        text=text.detach().numpy(), img=img.numpy(), text_mask=text_mask.numpy(),
        img_mask=(img_mask.numpy() if img_mask is not None else np.zeros((0,), bool)),
        img_keep=img_keep.numpy(), txt_keep=txt_keep.numpy(), attn_keep=attn_keep.numpy(),
        res=res.detach().numpy(), mask_out=mask_out.numpy(), gout=gout.numpy(),
        grad_text=text.grad.numpy(),
    )
    for k, v in h.named_parameters():
        out["param." + k] = v.detach().numpy()
        out["grad." + k] = (v.grad.numpy() if v.grad is not None else np.zeros_like(v.detach().numpy()))
    np.savez_compressed(os.path.join(OUT, f"fusion_{name}.npz"), **out)
    return res


def _make_external_case(F, name, *, d, Di, N, B, Te, Ti, text_pad, img_pad, seed=0):
    """The reference's ExternalMultimodalTransformerEncoder (fuse.py:288-357) exactly as
    MM_S2STransformerEncoder builds it for multimodal_attention_type
    "external_multimodal_transformer" (mm_s2s_transformer.py:156-171: TransformerLayerConfig(
    embed_dim=d, kdim=vdim=Di, nhead=Di // 64, dim_feedforward=4 Di, dropout, batch_first=False))
    and calls it (:531-554, :582-591: m1 = the last N encoder states, m2 = the image features
    expanded N times, key padding masks).  Dropout 0 (torch MHA's internal dropout cannot be
    replayed); train mode."""
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    cfgl = F.TransformerLayerConfig(embed_dim=d, kdim=Di, vdim=Di, nhead=Di // 64, dim_feedforward=Di * 4,
                                    dropout=0.0, batch_first=False)
    enc = F.ExternalMultimodalTransformerEncoder(layer_config=cfgl, num_layers=N)
    with torch.no_grad():
        for n, prm in enc.named_parameters():
            if n.endswith("bias"):
                prm.copy_(0.1 * torch.randn(prm.shape, generator=g))
            elif "norm" in n:
                prm.copy_(1.0 + 0.1 * torch.randn(prm.shape, generator=g))
    enc = enc.double().train()
    feats = [torch.randn(Te, B, d, generator=g, dtype=torch.float64).requires_grad_(True) for _ in range(N)]
    img = torch.randn(Ti, B, Di, generator=g, dtype=torch.float64)
    text_len = torch.full((B,), Te, dtype=torch.long)
    if text_pad:
        text_len = torch.randint(max(1, Te // 2), Te + 1, (B,), generator=g)
        text_len[0] = Te
    text_mask = torch.arange(Te)[None, :] >= text_len[:, None]
    img_mask = None
    if img_pad:
        img_len = torch.randint(max(1, Ti // 2), Ti + 1, (B,), generator=g)
        img_len[0] = Ti
        img_mask = torch.arange(Ti)[None, :] >= img_len[:, None]
    m2 = img.unsqueeze(0).expand(N, -1, -1, -1)   # mm_s2s_transformer.expand(img, N)
    res = enc(m1=feats, m2=m2, m1_mask=None, m2_mask=None, m1_key_padding_mask=text_mask,
              m2_key_padding_mask=img_mask)
    gout = torch.randn(res.shape, generator=g, dtype=torch.float64)
    (res * gout).sum().backward()
    out = dict(d=np.array(d), Di=np.array(Di), N=np.array(N), img=img.numpy(), text_mask=text_mask.numpy(),
               img_mask=(img_mask.numpy() if img_mask is not None else np.zeros((0,), bool)),
               res=res.detach().numpy(), gout=gout.numpy())
    for i, f in enumerate(feats):
        out[f"feat{i}"] = f.detach().numpy()
        out[f"grad_feat{i}"] = f.grad.numpy()
    for k, v in enc.named_parameters():
        out["param." + k] = v.detach().numpy()
        out["grad." + k] = (v.grad.numpy() if v.grad is not None else np.zeros_like(v.detach().numpy()))
    np.savez_compressed(os.path.join(OUT, f"external_{name}.npz"), **out)
    return res


def main():
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    os.makedirs(OUT, exist_ok=True)
    _install_shim()
    import mm_s2ut.models.fuse as F  # noqa: E402  (reference code, shimmed deps)
    import mm_s2ut.models.mm_s2s_transformer as M  # noqa: E402
    cases = [
        # name, attention, gate, d, Di, B, Te, Ti, text_pad, img_pad, dropout p's
        ("mma_gate_packed", "multimodal_attention", True, 64, 64, 3, 9, 17, True, False, 0, 0, 0),
        ("mma_gate_sep_imgmask", "multimodal_attention", True, 64, 96, 3, 9, 17, True, True, 0, 0, 0),
        ("mma_nogate", "multimodal_attention", False, 64, 64, 2, 7, 13, False, True, 0, 0, 0),
        ("sa_gate", "selective_attention", True, 64, 96, 3, 9, 17, True, False, 0, 0, 0),
        ("sa_gate_imgmask", "selective_attention", True, 64, 64, 3, 9, 17, True, True, 0, 0, 0),
        ("sa_nogate", "selective_attention", False, 32, 48, 2, 5, 11, False, False, 0, 0, 0),
        ("sa_gate_dropout", "selective_attention", True, 64, 96, 3, 9, 17, True, True, 0.3, 0.2, 0.1),
        ("mma_gate_dropout", "multimodal_attention", True, 64, 64, 2, 9, 17, True, False, 0.5, 0.1, 0),
        ("mma_gate_detr", "multimodal_attention", True, 96, 32, 2, 6, 10, True, True, 0, 0, 0),
    ]
    for i, (name, att, gate, d, Di, B, Te, Ti, tp, ip, pi, pt, pa) in enumerate(cases):
        _make_case(M, F, name, att=att, gate=gate, d=d, Di=Di, B=B, Te=Te, Ti=Ti,
                   text_pad=tp, img_pad=ip, p_img=pi, p_txt=pt, p_attn=pa, seed=100 + i)
        print("wrote", name)
    ext = [
        # name, d, Di, N layers, B, Te, Ti, text_pad, img_pad
        ("packed_2l", 64, 64, 2, 3, 9, 17, True, False),
        ("packed_3l_masks", 64, 64, 3, 2, 11, 13, True, True),
        ("heads2_2l", 64, 128, 2, 2, 6, 9, True, True),
        ("separate_2l", 96, 64, 2, 3, 7, 10, False, True),
    ]
    for i, (name, d, Di, N, B, Te, Ti, tp, ip) in enumerate(ext):
        _make_external_case(F, name, d=d, Di=Di, N=N, B=B, Te=Te, Ti=Ti, text_pad=tp, img_pad=ip, seed=200 + i)
        print("wrote external", name)


if __name__ == "__main__":
    main()
