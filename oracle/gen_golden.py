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


def _make_qformer_case(F, name, *, D, Q, nq, nm, B, Te, Ti, text_pad, sa_first, seed=0):
    """The reference's QFormerModel (fuse.py:769-874) as MM_S2STransformerEncoder builds it
    (mm_s2s_transformer.py:195-207: TransformerLayerConfig(embed_dim = kdim = vdim = D,
    nhead = D // 64, FFN 4 D, batch_first=True), self_attention_first from the config) and calls it
    (:481-486: m1 = encoder_out [B, Te, D] with its padding mask, m2 = image features [B, Ti, D],
    no image mask).  Dropout 0; train mode; query_embedding drawn nonzero.  Inputs and parameters
    are fp16-representable (the HIP run sees the same values); results are stored as float32."""
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    cfgl = F.TransformerLayerConfig(embed_dim=D, kdim=D, vdim=D, nhead=max(1, D // 64), dim_feedforward=4 * D,
                                    dropout=0.0, batch_first=True)
    qf = F.QFormerModel(num_queries=Q, layer_config=cfgl, num_query_layers=nq, num_multimodal_layers=nm,
                        self_attention_first=sa_first)
    with torch.no_grad():
        for n, prm in qf.named_parameters():
            if n == "query_embedding":
                prm.copy_(0.5 * torch.randn(prm.shape, generator=g))
            elif n.endswith("bias"):
                prm.copy_(0.1 * torch.randn(prm.shape, generator=g))
            elif "norm" in n:
                prm.copy_(1.0 + 0.1 * torch.randn(prm.shape, generator=g))
            prm.copy_(prm.half().float())
    qf = qf.double().train()
    m1 = torch.randn(B, Te, D, generator=g).half().double().requires_grad_(True)
    m2 = torch.randn(B, Ti, D, generator=g).half().double().requires_grad_(True)
    text_len = torch.full((B,), Te, dtype=torch.long)
    if text_pad:
        text_len = torch.randint(max(1, Te // 2), Te + 1, (B,), generator=g)
        text_len[0] = Te
    text_mask = torch.arange(Te)[None, :] >= text_len[:, None]
    res = qf(m1=m1, m2=m2, m1_key_padding_mask=text_mask, m2_key_padding_mask=None)
    gout = torch.randn(res.shape, generator=g).half().double()
    (res * gout).sum().backward()
    f32 = lambda t: t.detach().numpy().astype(np.float32)  # noqa: E731
    out = dict(D=np.array(D), Q=np.array(Q), nq=np.array(nq), nm=np.array(nm), sa_first=np.array(sa_first),
               m1=m1.detach().numpy().astype(np.float16), m2=m2.detach().numpy().astype(np.float16),
               text_mask=text_mask.numpy(), res=f32(res), gout=gout.numpy().astype(np.float16),
               grad_m1=f32(m1.grad), grad_m2=f32(m2.grad))
    for k, v in qf.named_parameters():
        out["param." + k] = v.detach().numpy().astype(np.float16)
        out["grad." + k] = f32(v.grad)
    np.savez_compressed(os.path.join(OUT, f"qformer_{name}.npz"), **out)
    return res


SHIPPED = dict(d=768, Di=768, B=2, Te=125, Ti=577, seed=300, probes=8)


def shipped_inputs(seed=SHIPPED["seed"]):
    """Inputs and parameters of the shipped-shape fusion golden case: d = Di =
    768 (packed in_proj), Ti = 577 ViT tokens (+ the bias_kv key = 578), Te = 125, B = 2, text and
    image padding.  Everything comes from a seeded numpy PCG64 stream and is rounded to fp16, so the
    reference's float64 run and the HIP fp16 run see identical values; the fixture stores a SHA-256
    of every array instead of the 3.5 M parameters (tests recompute and check it).  Weight
    gradients are stored as sketches G @ R and L^T @ G with the Gaussian probes returned here."""
    c = SHIPPED
    d, Di, B, Te, Ti = c["d"], c["Di"], c["B"], c["Te"], c["Ti"]
    rng = np.random.default_rng(seed)

    def h(x):
        return np.asarray(x, np.float16).astype(np.float64)

    def xavier(o, i):
        a = np.sqrt(6.0 / (i + o))
        return h(rng.uniform(-a, a, (o, i)))

    P = {
        "image_pre_norm_module.weight": h(1.0 + 0.1 * rng.standard_normal(Di)),
        "image_pre_norm_module.bias": h(0.1 * rng.standard_normal(Di)),
        "gate_denses.0.weight": xavier(d, 2 * d),
        "gate_denses.0.bias": h(0.1 * rng.standard_normal(d)),
        "in_proj_weight": np.concatenate([xavier(d, d) / np.sqrt(2), xavier(d, Di) / np.sqrt(2),
                                          xavier(d, Di) / np.sqrt(2)]).astype(np.float16).astype(np.float64),
        "in_proj_bias": h(0.1 * rng.standard_normal(3 * d)),
        "bias_k": h(0.05 * rng.standard_normal((1, 1, d))),
        "bias_v": h(0.05 * rng.standard_normal((1, 1, d))),
        "out_proj.weight": xavier(d, d),
        "out_proj.bias": h(0.1 * rng.standard_normal(d)),
    }
    X = {"text": h(rng.standard_normal((Te, B, d))), "img": h(rng.standard_normal((Ti, B, Di))),
         "gout": h(rng.standard_normal((Te, B, d)))}
    text_len = np.array([Te, 100])
    img_len = np.array([Ti, 450])
    X["text_mask"] = np.arange(Te)[None, :] >= text_len[:, None]
    X["img_mask"] = np.arange(Ti)[None, :] >= img_len[:, None]
    shapes = {"in_proj_weight": (3 * d, d), "out_proj.weight": (d, d), "gate_denses.0.weight": (d, 2 * d),
              "q_proj.weight": (d, d), "k_proj.weight": (d, Di), "v_proj.weight": (d, Di), "proj.weight": (d, d)}
    probes = {n: (rng.standard_normal((sh[1], c["probes"])), rng.standard_normal((sh[0], c["probes"])))
              for n, sh in shapes.items()}
    return P, X, probes


def shipped_model_params(P, att):
    """The shipped case's parameters under the model's state-dict names (``encoder.*``) for one
    attention type (selective attention takes q / k / v from the packed rows, proj = out_proj)."""
    d = SHIPPED["d"]
    out = {f"encoder.{k}": P[k] for k in ("image_pre_norm_module.weight", "image_pre_norm_module.bias",
                                          "gate_denses.0.weight", "gate_denses.0.bias")}
    if att == "multimodal_attention":
        for k in ("in_proj_weight", "in_proj_bias", "bias_k", "bias_v", "out_proj.weight", "out_proj.bias"):
            out[f"encoder.multimodal_attns.0.{k}"] = P[k]
        return out
    W, b = P["in_proj_weight"], P["in_proj_bias"]
    for j, n in enumerate("qkv"):
        out[f"encoder.selective_attns.0.{n}_proj.weight"] = W[j * d:(j + 1) * d]
        out[f"encoder.selective_attns.0.{n}_proj.bias"] = b[j * d:(j + 1) * d]
    out["encoder.selective_attns.0.proj.weight"] = P["out_proj.weight"]
    out["encoder.selective_attns.0.proj.bias"] = P["out_proj.bias"]
    return out


def array_digest(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(np.asarray(a, np.float16)).tobytes()).hexdigest()


def _make_shipped(M, F):
    """Both attention types at the shipped shape, gate on, dropout 0 (the HIP RNG's masks cannot be
    injected into nn.MultiheadAttention), float64 -> tests/golden/shipped_fusion.npz."""
    c = SHIPPED
    d, Di = c["d"], c["Di"]
    P, X, probes = shipped_inputs()
    out = {"seed": np.array(c["seed"]), **{f"digest.{k}": np.array(array_digest(v)) for k, v in {**P, **X}.items()
                                           if k not in ("text_mask", "img_mask")}}
    out["text_mask"], out["img_mask"] = X["text_mask"], X["img_mask"]
    T = lambda a: torch.from_numpy(np.array(a))  # noqa: E731
    for att in ("multimodal_attention", "selective_attention"):
        hm = nn.Module()
        hm.image_pre_norm_module = nn.LayerNorm([Di], 1e-5, True)
        hm.image_dropout_module = MaskDropout(0.0, None)
        hm.text_dropout_module = MaskDropout(0.0, None)
        hm.gate_denses = nn.ModuleList([M.Linear(2 * d, d)])
        hm.use_selective_gate, hm.is_merge_text_img, hm.multimodal_attention_type = True, False, att
        if att == "multimodal_attention":
            hm.multimodal_attns = nn.ModuleList([F.MultimodalAttention(embed_dim=d, kdim=Di, vdim=Di, num_heads=1,
                                                                       dropout=0.0, add_bias_kv=True)])
            names = {"multimodal_attns.0." + k: k for k in ("in_proj_weight", "in_proj_bias", "bias_k", "bias_v",
                                                           "out_proj.weight", "out_proj.bias")}
            src = dict(P)
        else:
            hm.selective_attns = nn.ModuleList([F.SelectiveAttention(qdim=d, kdim=Di, vdim=Di, attn_dim=d,
                                                                     intermediate_dim=d, output_dim=d, num_heads=1,
                                                                     attn_drop=0.0)])
            W, b = P["in_proj_weight"], P["in_proj_bias"]
            src = dict(P, **{"q_proj.weight": W[:d], "k_proj.weight": W[d:2 * d], "v_proj.weight": W[2 * d:],
                             "q_proj.bias": b[:d], "k_proj.bias": b[d:2 * d], "v_proj.bias": b[2 * d:],
                             "proj.weight": P["out_proj.weight"], "proj.bias": P["out_proj.bias"]})
            names = {"selective_attns.0." + k: k for k in ("q_proj.weight", "k_proj.weight", "v_proj.weight",
                                                          "q_proj.bias", "k_proj.bias", "v_proj.bias",
                                                          "proj.weight", "proj.bias")}
        names.update({k: k for k in ("image_pre_norm_module.weight", "image_pre_norm_module.bias",
                                     "gate_denses.0.weight", "gate_denses.0.bias")})
        hm = hm.double().train()
        with torch.no_grad():
            for n, prm in hm.named_parameters():
                prm.copy_(T(src[names[n]]).view(prm.shape))
        text = T(X["text"]).requires_grad_(True)
        res, _ = M.MM_S2STransformerEncoder.fuse_img_feat(hm, text, 0, T(X["img"]), T(X["img_mask"]),
                                                         T(X["text_mask"]))
        (res * T(X["gout"])).sum().backward()
        tag = "mma" if att == "multimodal_attention" else "sa"
        out[f"{tag}.res"] = res.detach().numpy().astype(np.float32)
        out[f"{tag}.grad_text"] = text.grad.numpy().astype(np.float32)
        for n, prm in hm.named_parameters():
            g = prm.grad.numpy().reshape(prm.shape)
            key = names[n]
            if g.ndim == 2:
                R_, L_ = probes[key]
                out[f"{tag}.gsk.{n}"] = (g @ R_).astype(np.float32)
                out[f"{tag}.gskT.{n}"] = (L_.T @ g).astype(np.float32)
            else:
                out[f"{tag}.grad.{n}"] = g.astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "shipped_fusion.npz"), **out)


def main():
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    os.makedirs(OUT, exist_ok=True)
    _install_shim()
    import mm_s2ut.models.fuse as F  # noqa: E402  (reference code, shimmed deps)
    import mm_s2ut.models.mm_s2s_transformer as M  # noqa: E402
    only = sys.argv[1:]    # e.g. "qformer": regenerate that family only
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
    for i, (name, att, gate, d, Di, B, Te, Ti, tp, ip, pi, pt, pa) in enumerate(cases if not only else []):
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
    for i, (name, d, Di, N, B, Te, Ti, tp, ip) in enumerate(ext if not only else []):
        _make_external_case(F, name, d=d, Di=Di, N=N, B=B, Te=Te, Ti=Ti, text_pad=tp, img_pad=ip, seed=200 + i)
        print("wrote external", name)
    qf = [
        # name, D, queries, query layers, multimodal layers, B, Te, Ti, text_pad, self_attention_first
        ("d64_2q1m", 64, 5, 2, 1, 3, 9, 7, True, False),
        ("d128_1q1m_safirst", 128, 4, 1, 1, 2, 11, 6, True, True),
        ("d64_1q2m", 64, 8, 1, 2, 2, 13, 17, False, False),
    ]
    if not only or "qformer" in only:
        for i, (name, D, Q, nq, nm, B, Te, Ti, tp, saf) in enumerate(qf):
            _make_qformer_case(F, name, D=D, Q=Q, nq=nq, nm=nm, B=B, Te=Te, Ti=Ti, text_pad=tp, sa_first=saf,
                               seed=400 + i)
            print("wrote qformer", name)
    if not only:
        _make_shipped(M, F)
        print("wrote shipped_fusion")


if __name__ == "__main__":
    main()
