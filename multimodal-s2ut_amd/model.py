"""MI355X-native mm_s2ut_transformer: parameters, forward and hand-written backward.

The model is restated MI355X-first: all activations are batch-major ``[B*T, C]`` fp16 rows in HBM,
every op is a libmms2ut_hip kernel (MFMA GEMMs with fused epilogues, wave-reduction LayerNorm /
softmax, counter-RNG dropout), and the backward pass is written out by hand per layer (no
autograd tape inside the model).  Parameters live in ONE flat fp16 buffer whose layout is the
backward-completion order, so gradient buckets become ready front-to-back during backward
(RCCL all-reduce overlap, see parallel.py).  Key names are those of the reference's
``MM_S2UTTransformerModel.state_dict()`` (fairseq module tree) so checkpoints interchange.

Reference path restated here:
  MM_S2UTTransformerModel.forward            mm_s2ut/models/mm_s2s_transformer.py:667-700
  MM_S2STransformerEncoder.forward           mm_s2s_transformer.py:378-562 (default S2T branch)
    fairseq S2TTransformerEncoder._forward   (Conv1dSubsampler, sinusoidal pos, 12 pre-LN layers)
    fusion tail                              mm_s2s_transformer.py:471-560
    fuse_img_feat                            mm_s2s_transformer.py:594-622
    SelectiveAttention / MultimodalAttention mm_s2ut/models/fuse.py:35-117 / 120-167
  fairseq TransformerUnitDecoder             (6 pre-LN layers, tied output projection)
"""
import math
import os
import re
from collections import OrderedDict

import numpy as np
import torch

from . import kernels as K
from .kernels import F16, round_up

# ============================================================================ config


def default_cfg(**over):
    """`s2ut_architecture_base` + textless/1_train.sh flags + shipped fusion YAML
    (mm_s2ut/config/multimodal_s2ut_transformer.yaml)."""
    cfg = dict(
        input_feat_per_channel=80, input_channels=1, conv_kernel_sizes=(5, 5), conv_channels=1024,
        encoder_embed_dim=768, encoder_ffn_embed_dim=3072, encoder_layers=12,
        encoder_attention_heads=8, decoder_embed_dim=768, decoder_ffn_embed_dim=3072,
        decoder_layers=6, decoder_attention_heads=8, dropout=0.1, attention_dropout=0.1,
        activation_dropout=0.1, vocab_size=1004, padding_idx=1, eos=2, label_smoothing=0.2,
        fusion=True, multimodal_attention_type="multimodal_attention", use_selective_gate=True,
        image_feat_dim=768, image_pre_norm=True, SA_image_dropout=0.1, SA_text_dropout=0.0,
        SA_attention_dropout=0.1, modality_dropout=-0.5, audio_dropout=-0.5,
        max_source_positions=6000, max_target_positions=3000, no_scale_embedding=False,
        external_multimodal_transformer_layers=None,
        # QFormer extractor (mm_s2s_transformer.py:194-209; multimodal_translation_config keys)
        multimodal_extractor_type=None, num_queries=32, num_query_layers=4, num_multimodal_layers=2,
        self_attention_first=False,
    )
    cfg.update(over)
    return cfg

# ============================================================================ decoder specs


class DecoderSpec:
    """One fairseq TransformerDecoder (pre-LN, sinusoidal positions, tied output projection) over
    the flat parameter buffer: the unit decoder (prefix "decoder") or a multitask auxiliary
    transformer decoder (prefix "{task}_decoder", fairseq S2STransformerMultitaskModelBase;
    base_multitask_text_transformer_decoder_arch dims).  kdim: the encoder dim it cross-attends."""

    def __init__(self, prefix, d, H, F, L, V, kdim, dropout, attention_dropout, activation_dropout,
                 pad=1, no_scale_embedding=False, max_target_positions=3000):
        self.prefix, self.d, self.H, self.F, self.L, self.V, self.kdim = prefix, d, H, F, L, V, kdim
        self.pd, self.pa, self.pact = dropout, attention_dropout, activation_dropout
        self.pad, self.no_scale_embedding, self.max_target_positions = pad, no_scale_embedding, max_target_positions

    @classmethod
    def main(cls, cfg):
        return cls("decoder", cfg["decoder_embed_dim"], cfg["decoder_attention_heads"], cfg["decoder_ffn_embed_dim"],
                   cfg["decoder_layers"], cfg["vocab_size"], cfg["encoder_embed_dim"], cfg["dropout"],
                   cfg["attention_dropout"], cfg["activation_dropout"], cfg["padding_idx"],
                   cfg["no_scale_embedding"], cfg["max_target_positions"])

    @classmethod
    def aux(cls, cfg, t):
        """A multitask task dict (multitask.task_model_cfg) of decoder_type transformer."""
        return cls(f"{t['name']}_decoder", t["d"], t["H"], t["F"], t["L"], t["V"], cfg["encoder_embed_dim"],
                   t["dropout"], t["attention_dropout"], t["activation_dropout"], t["pad"],
                   t.get("no_scale_embedding", False), t.get("max_target_positions", 1024))


def aux_tasks(cfg):
    return list(cfg.get("multitask") or [])


def _decoder_param_specs(S, spec, mha, ln):
    """Backward-completion order of one decoder: final LN, layers L-1..0, the layer-major
    cross-attention K/V slab, the (tied) token embedding."""
    p0, dd, Fd = spec.prefix, spec.d, spec.F
    ln(f"{p0}.layer_norm", dd)
    for l in reversed(range(spec.L)):
        p = f"{p0}.layers.{l}"
        S.extend([(f"{p}.fc2.weight", (dd, Fd)), (f"{p}.fc2.bias", (dd,)),
                  (f"{p}.fc1.weight", (Fd, dd)), (f"{p}.fc1.bias", (Fd,))])
        ln(p + ".final_layer_norm", dd)
        mha(p + ".encoder_attn", dd, spec.kdim, kv=False)
        ln(p + ".encoder_attn_layer_norm", dd)
        mha(p + ".self_attn", dd, dd)
        ln(p + ".self_attn_layer_norm", dd)
    # Every layer's cross-attention K/V projection reads the same encoder output, so their
    # weights sit layer-major in one [L*2*dd, kdim] slab (and biases in one [L*2*dd] vector): one
    # forward GEMM, one dgrad and one wgrad for all layers.  Their gradients complete after the
    # whole decoder backward, hence the block's place after the layers.
    for l in range(spec.L):
        p = f"{p0}.layers.{l}.encoder_attn"
        S.extend([(f"{p}.k_proj.weight", (dd, spec.kdim)), (f"{p}.v_proj.weight", (dd, spec.kdim))])
    for l in range(spec.L):
        p = f"{p0}.layers.{l}.encoder_attn"
        S.extend([(f"{p}.k_proj.bias", (dd,)), (f"{p}.v_proj.bias", (dd,))])
    S.append((f"{p0}.embed_tokens.weight", (spec.V, dd)))

EXT = "encoder.multimodal_transformer.0"
# parameters of the fusion tail (mm_s2s_transformer.py:471-622) and its image-side extractors
FUSION_PREFIXES = ("encoder.gate", "encoder.multimodal", "encoder.selective", "encoder.image", "encoder.q_former")


def external_dims(cfg):
    """(d, Di, heads, head dim, FFN, layers) of the external transformer as the reference builds it
    (mm_s2s_transformer.py:156-171: kdim = vdim = Di, nhead = Di // 64, FFN 4 Di)."""
    d, Di = cfg["encoder_embed_dim"], cfg["image_feat_dim"]
    N = cfg["external_multimodal_transformer_layers"]
    if not N or N < 1 or N > cfg["encoder_layers"]:
        raise ValueError(f"external_multimodal_transformer_layers={N!r} (1..encoder_layers)")
    H = Di // 64
    if H < 1 or d % H:
        raise NotImplementedError(f"external transformer: nhead = Di // 64 = {H} must divide embed_dim {d}")
    return d, Di, H, d // H, 4 * Di, N


def _external_param_specs(S, cfg, ln):
    """ExternalMultimodalTransformerEncoder (fuse.py:288-357) parameter names / shapes, layers in
    backward-completion order, the shared layer_norm1 last."""
    d, Di, H, hd, F_, N = external_dims(cfg)
    for i in reversed(range(N)):
        _mml_param_specs(S, f"{EXT}.layers.{i}", d, Di, F_, ln)
    ln(EXT + ".layer_norm1", d)

QF = "encoder.q_former"


def qformer_dims(cfg, check=True):
    """(D, heads, FFN, queries, query layers, multimodal layers, self_attention_first) of the
    QFormerModel built at mm_s2s_transformer.py:195-207 (TransformerLayerConfig(embed_dim = kdim =
    vdim = 768, nhead = 768 // 64, FFN 4·768)): the width is the image feature width (768 for ViT)
    and must equal encoder_embed_dim, since the query layers attend to the encoder output."""
    D, d = cfg["image_feat_dim"], cfg["encoder_embed_dim"]
    if check and D != d:
        raise NotImplementedError(f"q_former: width {D} (image_feat_dim) must equal encoder_embed_dim {d}")
    H = max(1, D // 64)
    if check and (D % H or (D // H) not in K.FLASH_HD):
        raise NotImplementedError(f"q_former: head dim {D // H} not supported")
    return (D, H, 4 * D, cfg["num_queries"], cfg["num_query_layers"], cfg["num_multimodal_layers"],
            bool(cfg["self_attention_first"]))


def _mml_param_specs(S, p, d, kdim, F_, ln, sa_first=True):
    """One MultimodalTransformerDecoderLayer (fuse.py:187-221), backward-completion order."""
    S.extend([(p + ".linear2.weight", (d, F_)), (p + ".linear2.bias", (d,)),
              (p + ".linear1.weight", (F_, d)), (p + ".linear1.bias", (F_,))])
    ln(p + ".norm3", d)

    def ca():
        ln(p + ".norm2", d)
        S.extend([(p + ".multihead_attn.out_proj.weight", (d, d)), (p + ".multihead_attn.out_proj.bias", (d,))])
        if kdim == d:
            S.append((p + ".multihead_attn.in_proj_weight", (3 * d, d)))
        else:
            S.extend([(p + ".multihead_attn.q_proj_weight", (d, d)), (p + ".multihead_attn.k_proj_weight", (d, kdim)),
                      (p + ".multihead_attn.v_proj_weight", (d, kdim))])
        S.append((p + ".multihead_attn.in_proj_bias", (3 * d,)))

    def sa():
        ln(p + ".norm1", d)
        S.extend([(p + ".self_attn.out_proj.weight", (d, d)), (p + ".self_attn.out_proj.bias", (d,)),
                  (p + ".self_attn.in_proj_weight", (3 * d, d)), (p + ".self_attn.in_proj_bias", (3 * d,))])

    if sa_first:
        ca()
        sa()
    else:
        sa()
        ca()


def _qformer_param_specs(S, cfg, ln, check=True):
    """QFormerModel (fuse.py:769-818): multimodal layers then query layers in backward order, the
    query embedding last."""
    D, _, F_, Q, nq, nm, saf = qformer_dims(cfg, check)
    for i in reversed(range(nm)):
        _mml_param_specs(S, f"{QF}.multimodal_transformer_layers.{i}", D, D, F_, ln, saf)
    for i in reversed(range(nq)):
        _mml_param_specs(S, f"{QF}.query_transformer_layers.{i}", D, D, F_, ln, saf)
    S.append((QF + ".query_embedding", (1, Q, D)))

# ============================================================================ parameter layout


def param_specs(cfg):
    """Ordered (name, shape) list in backward-completion order + the never-used params (Q3)."""
    d, F_, C = cfg["encoder_embed_dim"], cfg["encoder_ffn_embed_dim"], cfg["conv_channels"]
    dd, Fd, V = cfg["decoder_embed_dim"], cfg["decoder_ffn_embed_dim"], cfg["vocab_size"]
    cin = cfg["input_feat_per_channel"] * cfg["input_channels"]
    ks = cfg["conv_kernel_sizes"]
    S = []

    def mha(p, dm, kd, kv=True):
        # q, k, v adjacent (fused QKV / KV GEMMs), then biases q, k, v adjacent; kv=False leaves
        # k/v to the decoder's cross-attention block below
        S.append((f"{p}.q_proj.weight", (dm, dm)))
        if kv:
            S.extend([(f"{p}.k_proj.weight", (dm, kd)), (f"{p}.v_proj.weight", (dm, kd))])
        S.append((f"{p}.q_proj.bias", (dm,)))
        if kv:
            S.extend([(f"{p}.k_proj.bias", (dm,)), (f"{p}.v_proj.bias", (dm,))])
        S.extend([(f"{p}.out_proj.weight", (dm, dm)), (f"{p}.out_proj.bias", (dm,))])

    def ln(p, n):
        S.extend([(f"{p}.weight", (n,)), (f"{p}.bias", (n,))])

    tasks = aux_tasks(cfg)
    qf_unused = []
    # multitask heads on the unit decoder's inner states complete their backward first, then the
    # unit decoder, then the heads on encoder states, then the encoder (runtime._ModelFn.backward)
    for t in tasks:
        if t["type"] == "ctc" and t["input_from"] == "decoder":
            S.extend([(f"{t['name']}_decoder.proj.weight", (t["V"], dd)), (f"{t['name']}_decoder.proj.bias", (t["V"],))])
    _decoder_param_specs(S, DecoderSpec.main(cfg), mha, ln)
    for t in tasks:
        if t["type"] == "transformer":
            _decoder_param_specs(S, DecoderSpec.aux(cfg, t), mha, ln)
        elif t["input_from"] == "encoder":
            S.extend([(f"{t['name']}_decoder.proj.weight", (t["V"], d)), (f"{t['name']}_decoder.proj.bias", (t["V"],))])
    ext = cfg["fusion"] and cfg["multimodal_attention_type"] == "external_multimodal_transformer"
    if cfg["fusion"] and not ext:
        S.extend([("encoder.gate_denses.0.weight", (d, 2 * d)), ("encoder.gate_denses.0.bias", (d,))])
    if cfg["fusion"]:
        Di = cfg["image_feat_dim"]
        if cfg["multimodal_attention_type"] == "multimodal_attention":
            p = "encoder.multimodal_attns.0"
            S.extend([(p + ".out_proj.weight", (d, d)), (p + ".out_proj.bias", (d,))])
            if Di == d:
                S.append((p + ".in_proj_weight", (3 * d, d)))
            else:
                S.extend([(p + ".q_proj_weight", (d, d)), (p + ".k_proj_weight", (d, Di)),
                          (p + ".v_proj_weight", (d, Di))])
            S.extend([(p + ".in_proj_bias", (3 * d,)), (p + ".bias_k", (1, 1, d)),
                      (p + ".bias_v", (1, 1, d))])
        elif cfg["multimodal_attention_type"] == "external_multimodal_transformer":
            _external_param_specs(S, cfg, ln)
        elif cfg["multimodal_attention_type"] == "selective_attention":
            p = "encoder.selective_attns.0"
            S.extend([(p + ".proj.weight", (d, d)), (p + ".proj.bias", (d,)),
                      (p + ".q_proj.weight", (d, d)), (p + ".k_proj.weight", (d, Di)),
                      (p + ".v_proj.weight", (d, Di)), (p + ".q_proj.bias", (d,)),
                      (p + ".k_proj.bias", (d,)), (p + ".v_proj.bias", (d,))])
        else:
            raise NotImplementedError(cfg["multimodal_attention_type"])
        if cfg["image_pre_norm"] and not ext:
            ln("encoder.image_pre_norm_module", Di)
        if not ext and cfg["multimodal_extractor_type"] == "q_former":
            _qformer_param_specs(S, cfg, ln)
        elif not ext and cfg.get("qformer_unused"):
            # built by the reference without a visual extractor, never called (mm_s2s_transformer.py:475)
            _qformer_param_specs(qf_unused, cfg, lambda p, n: qf_unused.extend([(f"{p}.weight", (n,)), (f"{p}.bias", (n,))]),
                                 check=False)
    ln("encoder.layer_norm", d)
    for l in reversed(range(cfg["encoder_layers"])):
        p = f"encoder.transformer_layers.{l}"
        S.extend([(f"{p}.fc2.weight", (d, F_)), (f"{p}.fc2.bias", (d,)),
                  (f"{p}.fc1.weight", (F_, d)), (f"{p}.fc1.bias", (F_,))])
        ln(p + ".final_layer_norm", d)
        mha(p + ".self_attn", d, d)
        ln(p + ".self_attn_layer_norm", d)
    for i in reversed(range(len(ks))):
        ci = cin if i == 0 else C // 2
        co = C if i < len(ks) - 1 else 2 * d
        S.extend([(f"encoder.subsample.conv_layers.{i}.weight", (co, ci, ks[i])),
                  (f"encoder.subsample.conv_layers.{i}.bias", (co,))])
    unused = qf_unused + [("encoder.proj_768_to_512.weight", (512, 768)), ("encoder.proj_768_to_512.bias", (512,)),
              ("encoder.proj_1024_to_512.weight", (512, 1024)), ("encoder.proj_1024_to_512.bias", (512,)),
              ("encoder.proj_1024_to_768.weight", (768, 1024)), ("encoder.proj_1024_to_768.bias", (768,))]
    for j in range(3):
        unused.extend([(f"encoder.wav2vec2_adaptor.layers.{j}.weight", (1536, 1024 if j == 0 else 768, 3)),
                       (f"encoder.wav2vec2_adaptor.layers.{j}.bias", (1536,))])
    unused.extend([("encoder.wav2vec2_adaptor.layernorm.weight", (1024,)),
                   ("encoder.wav2vec2_adaptor.layernorm.bias", (1024,))])
    if ext:
        # built by the reference for every fusion type but unused by the external transformer
        # (mm_s2s_transformer.py:173-190): kept in the state dict, never computed (as Q3)
        unused.extend([("encoder.gate_denses.0.weight", (d, 2 * d)), ("encoder.gate_denses.0.bias", (d,))])
        if cfg["image_pre_norm"]:
            Di = cfg["image_feat_dim"]
            unused.extend([("encoder.image_pre_norm_module.weight", (Di,)), ("encoder.image_pre_norm_module.bias", (Di,))])
    return S, unused


class ParamStore:
    """One flat fp16 parameter buffer + one flat fp16 gradient buffer with per-name views."""

    ALIGN = 8  # elements (16 B) per parameter start: vector loads; keeps q|k|v spans contiguous

    def __init__(self, specs, device, unused=()):
        self.specs = list(specs)
        self.offsets = OrderedDict()
        off = 0
        for name, shape in self.specs:
            n = int(np.prod(shape))
            self.offsets[name] = (off, tuple(shape), n)
            off = round_up(off + n, self.ALIGN)
        self.numel = off
        self.flat = torch.zeros(self.numel, dtype=F16, device=device)
        self.grad = torch.zeros(self.numel, dtype=F16, device=device)
        self.unused = OrderedDict((n, torch.zeros(s, dtype=F16, device=device)) for n, s in unused)
        self.p = {k: self.view(k) for k in self.offsets}
        self.g = {k: self.view(k, grad=True) for k in self.offsets}
        self.groups = self._forward_groups()
        self.pending = {}   # group -> event of its (deferred) optimizer update, see await_group
        # The backward writes every gradient outright (or zeroes the ones a branch skips), so the
        # trainer never clears this buffer; True restores a per-micro-batch fill (A/B, tests).
        self.zero_each_step = os.environ.get("MMS2UT_GRAD_ZERO") == "1"

    @staticmethod
    def group_of(name):
        """Forward-consumption group of a parameter (one flat contiguous range per group)."""
        m = re.match(r"encoder\.transformer_layers\.(\d+)\.", name)
        if m:
            return f"enc{m.group(1)}"
        if name.startswith("encoder.subsample."):
            return "sub"
        if name.startswith("encoder."):
            return "enc_tail"        # final encoder LN + fusion
        if re.match(r"decoder\.layers\.\d+\.encoder_attn\.[kv]_proj\.", name):
            return "cross_kv"
        m = re.match(r"decoder\.layers\.(\d+)\.", name)
        if m:
            return f"dec{m.group(1)}"
        if name.startswith("decoder.embed_tokens"):
            return "dec_emb"
        m = re.match(r"(\w+)_decoder\.", name)
        if m:
            return f"aux_{m.group(1)}"     # a multitask head (one contiguous group per task)
        return "dec_ln"

    def _forward_groups(self):
        """[(group, start, end)] flat element ranges in the order the forward consumes them (the
        reverse of the backward-completion layout)."""
        runs = []
        for name, _ in self.specs:
            off, _, n = self.offsets[name]
            grp = self.group_of(name)
            if runs and runs[-1][0] == grp:
                runs[-1][2] = round_up(off + n, self.ALIGN)
            else:
                assert all(r[0] != grp for r in runs), f"group {grp} not contiguous"
                runs.append([grp, off, round_up(off + n, self.ALIGN)])
        runs[-1][2] = self.numel
        return [tuple(r) for r in reversed(runs)]

    def await_group(self, grp):
        """Make the current stream wait for a deferred optimizer update of `grp` (no-op if none)."""
        ev = self.pending.pop(grp, None)
        if ev is not None:
            ev.wait(torch.cuda.current_stream(self.flat.device))

    def await_all(self):
        for grp in list(self.pending):
            self.await_group(grp)

    def view(self, name, grad=False):
        off, shape, n = self.offsets[name]
        buf = self.grad if grad else self.flat
        return buf[off:off + n].view(shape)

    def span(self, first, last, grad=False):
        """Contiguous flat view from param `first` through `last` (inclusive)."""
        a = self.offsets[first][0]
        b = self.offsets[last][0] + self.offsets[last][2]
        buf = self.grad if grad else self.flat
        return buf[a:b]

    def load_state_dict(self, sd, strict=True):
        self.await_all()
        seen = set()
        for k, v in sd.items():
            if k in self.offsets:
                self.p[k].copy_(v.to(self.p[k].dtype).view(self.p[k].shape))
                seen.add(k)
            elif k in self.unused:
                self.unused[k].copy_(v.view(self.unused[k].shape))
                seen.add(k)
        missing = [k for k in self.offsets if k not in seen]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:5]}...")
        return missing

    def state_dict(self):
        self.await_all()
        sd = OrderedDict((k, v.detach().clone()) for k, v in self.p.items())
        for k, v in self.unused.items():
            sd[k] = v.detach().clone()
        sd["decoder.output_projection.weight"] = sd["decoder.embed_tokens.weight"]
        return sd


def sinusoidal_table(num, dim, padding_idx=1):
    """fairseq SinusoidalPositionalEmbedding.get_embedding (host constant, fp32 -> fp16)."""
    half = dim // 2
    emb = math.log(10000) / (half - 1)
    emb = torch.exp(torch.arange(half, dtype=torch.float) * -emb)
    emb = torch.arange(num, dtype=torch.float).unsqueeze(1) * emb.unsqueeze(0)
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=1).view(num, -1)
    if dim % 2 == 1:
        emb = torch.cat([emb, torch.zeros(num, 1)], dim=1)
    emb[padding_idx, :] = 0
    return emb

# ============================================================================ attention core


class AttnCtx:
    """What an attention forward saves for its backward (flash: lse; unfused: P, Pd)."""
    __slots__ = ("flash", "P", "Pd", "ldS", "lse", "key_len", "causal")


def attn_forward(q, k, v, ldq, ldk, ldv, B, H, Tq, Tk, hd, scale, out, ldo, *, key_len=None,
                 key_mask=None, causal=False, extra_key=False, p=0.0, drop=None):
    ctx = AttnCtx()
    ctx.key_len, ctx.causal = key_len, causal
    ctx.flash = key_mask is None and not extra_key and hd in K.FLASH_HD
    if ctx.flash:
        ctx.lse = K.mha_fwd(q, k, v, out, ldq, ldk, ldv, ldo, B, H, Tq, Tk, hd, scale, key_len=key_len,
                            causal=causal, p=p, drop=drop)
        ctx.P = ctx.Pd = None
        ctx.ldS = 0
    else:
        ctx.P, ctx.Pd, ctx.ldS = attn_fwd(q, k, v, ldq, ldk, ldv, B, H, Tq, Tk, hd, scale, out, ldo,
                                          key_len=key_len, key_mask=key_mask, causal=causal,
                                          extra_key=extra_key, p=p, drop=drop)
        ctx.lse = None
    return ctx


def attn_backward(ctx, dO, ldo, o, q, k, v, ldq, ldk, ldv, B, H, Tq, Tk, hd, scale, dq, dk, dv,
                  lddq, lddk, lddv, *, p=0.0, drop=None):
    if ctx.flash:
        K.mha_bwd(q, k, v, o, ldq, ldk, ldv, ldo, B, H, Tq, Tk, hd, scale, ctx.key_len, ctx.causal, p,
                  drop, ctx.lse, dO, ldo, dq, lddq, dk, lddk, dv, lddv)
    else:
        attn_bwd(dO, ldo, q, k, v, ldq, ldk, ldv, ctx.P, ctx.Pd, ctx.ldS, B, H, Tq, Tk, hd, scale, dq, dk,
                 dv, lddq, lddk, lddv, p=p, drop=drop)


def attn_fwd(q, k, v, ldq, ldk, ldv, B, H, Tq, Tk, hd, scale, out, ldo, *, key_len=None,
             key_mask=None, causal=False, extra_key=False, p=0.0, drop=None,
             sq=None, sk=None, so=None):
    """softmax(scale*q k^T + masks) -> dropout -> @ v, batched over (b, h), scores materialised.
    q/k/v/out are views whose row r=(b*T + t) and head column offset h*hd; `s*` = batch strides."""
    ldS = round_up(Tk, 8)
    sq = sq or Tq * ldq
    sk = sk or Tk * ldk
    so = so or Tq * ldo
    S = torch.empty(B * H * Tq * ldS, dtype=F16, device=q.device)
    K.gemm(q, k, S, Tq, Tk, hd, lda=ldq, ldb=ldk, ldc=ldS, batch=B * H, bdiv=H,
           sA=(sq, hd), sB=(sk, hd), sC=(H * Tq * ldS, Tq * ldS), alpha=scale)
    P, Pd = K.attn_softmax(S, B * H, H, Tq, Tk, ldS, key_len=key_len, key_mask=key_mask,
                           causal=causal, extra_key=extra_key, p=p, drop=drop)
    del S
    K.gemm(Pd, v, out, Tq, hd, Tk, a_kc=True, b_kc=False, lda=ldS, ldb=ldv, ldc=ldo, batch=B * H,
           bdiv=H, sA=(H * Tq * ldS, Tq * ldS), sB=(Tk * ldv if sk is None else sk, hd), sC=(so, hd))
    return P, Pd, ldS


def attn_bwd(dO, ldo, q, k, v, ldq, ldk, ldv, P, Pd, ldS, B, H, Tq, Tk, hd, scale, dq, dk, dv,
             lddq, lddk, lddv, *, p=0.0, drop=None, sq=None, sk=None, so=None, sdq=None, sdk=None):
    sq = sq or Tq * ldq
    sk = sk or Tk * ldk
    so = so or Tq * ldo
    sdq = sdq or Tq * lddq
    sdk = sdk or Tk * lddk
    sS = (H * Tq * ldS, Tq * ldS)
    dPd = torch.empty_like(P)
    # dPd = dO v^T
    K.gemm(dO, v, dPd, Tq, Tk, hd, lda=ldo, ldb=ldv, ldc=ldS, batch=B * H, bdiv=H,
           sA=(so, hd), sB=(sk, hd), sC=sS)
    # dv = Pd^T dO
    K.gemm(Pd, dO, dv, Tk, hd, Tq, a_kc=False, b_kc=False, lda=ldS, ldb=ldo, ldc=lddv,
           batch=B * H, bdiv=H, sA=sS, sB=(so, hd), sC=(sdk, hd))
    dS = K.attn_softmax_bwd(P, dPd, B * H, H, Tq, Tk, ldS, p=p, drop=drop)
    # dq = scale * dS k
    K.gemm(dS, k, dq, Tq, hd, Tk, a_kc=True, b_kc=False, lda=ldS, ldb=ldk, ldc=lddq,
           batch=B * H, bdiv=H, sA=sS, sB=(sk, hd), sC=(sdq, hd), alpha=scale)
    # dk = scale * dS^T q
    K.gemm(dS, q, dk, Tk, hd, Tq, a_kc=False, b_kc=False, lda=ldS, ldb=ldq, ldc=lddk,
           batch=B * H, bdiv=H, sA=sS, sB=(sq, hd), sC=(sdk, hd), alpha=scale)

# ============================================================================ the model


class MMS2UTModel:
    """Parameters + explicit forward/backward of MM_S2UTTransformerModel on one GPU."""

    def __init__(self, cfg, device="cuda", seed=1):
        self.cfg = cfg
        self.device = torch.device(device)
        specs, unused = param_specs(cfg)
        self.params = ParamStore(specs, self.device, unused)
        self.drop = K.Dropout(seed)
        self.training = True
        d, dd = cfg["encoder_embed_dim"], cfg["decoder_embed_dim"]
        self.enc_pos = sinusoidal_table(cfg["max_source_positions"] + 2, d).to(self.device, F16)
        self.dec_pos = sinusoidal_table(cfg["max_target_positions"] + 2, dd).to(self.device, F16)
        self.dspec = DecoderSpec.main(cfg)
        self.aux_specs = {t["name"]: DecoderSpec.aux(cfg, t) for t in aux_tasks(cfg) if t["type"] == "transformer"}
        self._pos = {}   # sinusoidal tables of other widths (multitask decoders)
        self.retain_tables = False   # graph mode: grown tables retire the old one (graphs bake it)
        self._retired = []
        self.np_rng = np.random  # modality-dropout draws use the global numpy stream (reference)
        # autograd anchor: the model's output is connected to the graph through this leaf
        self.anchor = torch.zeros(1, device=self.device, requires_grad=True)
        self.wt = None  # K.TransposedWeights of the dgrad weights (built at the first training forward)
        self._wpad = {}  # subsampler conv weights zero-padded to whole 64-wide k-tiles (subsample_fwd)
        self._layer_calls = {}  # layer prefix -> K.LayerCall (one-call transformer layers)
        self._conv = None       # K.ConvCall (one-call subsampler)
        self._fusion = {}       # image feature width -> K.FusionCall (one-call fusion tail)

    def dgrad_weights(self):
        """Every weight matrix the hand-written backward multiplies a gradient by (dx = dy @ W),
        exactly as the backward passes it to K.linear_dgrad."""
        cfg, P, span = self.cfg, self.P, self.params.span
        d, dd = cfg["encoder_embed_dim"], cfg["decoder_embed_dim"]
        mats = []

        def layer(p, dm):
            mats.extend([P(p + ".fc2.weight"), P(p + ".fc1.weight"), P(p + ".self_attn.out_proj.weight"),
                         span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight").view(3 * dm, dm)])

        for l in range(cfg["encoder_layers"]):
            layer(f"encoder.transformer_layers.{l}", d)
        for sp in [self.dspec] + list(self.aux_specs.values()):
            for l in range(sp.L):
                p = f"{sp.prefix}.layers.{l}"
                layer(p, sp.d)
                mats.extend([P(p + ".encoder_attn.out_proj.weight"), P(p + ".encoder_attn.q_proj.weight")])
            mats.append(self.cross_kv(spec=sp)[0])
        for i in range(1, len(cfg["conv_kernel_sizes"])):
            W = P(f"encoder.subsample.conv_layers.{i}.weight")
            mats.append(W.view(W.shape[0], -1))
        def mml(p, kdim, dmem):
            Wq, Wkv, _, _ = self._mha_w(p + ".multihead_attn", d, kdim)
            mats.extend([P(p + ".linear2.weight"), P(p + ".linear1.weight"), P(p + ".multihead_attn.out_proj.weight"),
                         Wq, P(p + ".self_attn.out_proj.weight"), P(p + ".self_attn.in_proj_weight")])
            if dmem:
                mats.append(Wkv)

        if cfg["fusion"] and cfg["multimodal_attention_type"] == "external_multimodal_transformer":
            for i in range(cfg["external_multimodal_transformer_layers"]):
                mml(f"{EXT}.layers.{i}", cfg["image_feat_dim"], False)
        elif cfg["fusion"]:
            if cfg.get("multimodal_extractor_type") == "q_former":
                D, _, _, _, nq, nm, _ = qformer_dims(cfg)
                for i in range(nq):
                    mml(f"{QF}.query_transformer_layers.{i}", D, True)
                for i in range(nm):
                    mml(f"{QF}.multimodal_transformer_layers.{i}", D, False)
            Di = cfg["image_feat_dim"]
            mats.append(P("encoder.gate_denses.0.weight"))
            if cfg["multimodal_attention_type"] == "multimodal_attention":
                pre = "encoder.multimodal_attns.0"
                mats.append(P(pre + ".out_proj.weight"))
                if Di == d:
                    W = P(pre + ".in_proj_weight")
                    mats.extend([W[:d], W[d:]])
                else:
                    mats.extend([P(pre + ".q_proj_weight"),
                                 span(pre + ".k_proj_weight", pre + ".v_proj_weight").view(2 * d, Di)])
            else:
                pre = "encoder.selective_attns.0"
                mats.extend([P(pre + ".proj.weight"), P(pre + ".q_proj.weight"),
                             span(pre + ".k_proj.weight", pre + ".v_proj.weight").view(2 * d, Di)])
        return [W for W in mats if W.shape[0] % 8 == 0 and W.shape[1] % 8 == 0]

    def refresh_transposed_weights(self):
        """Re-transpose the dgrad weights (side stream) for this step's backward."""
        if not (self.training and self.params.flat.is_cuda):
            K.TransposedWeights.active = None
            return
        if self.wt is None:
            self.wt = K.TransposedWeights(self.params.flat, self.dgrad_weights())
        self.wt.refresh()
        K.TransposedWeights.active = self.wt

    def init_params(self, seed=1):
        """Random init with fairseq's schemes (random-init weights of the architecture; no
        checkpoints are reachable offline): xavier for attention projections (gain 1/sqrt(2) for
        q/k/v), nn.Linear default for FFN/conv, N(0, d^-0.5) embedding with a zero pad row,
        LayerNorm (1, 0), zero biases for out_proj."""
        g = torch.Generator().manual_seed(seed)
        sd = {}
        for name, shape in self.params.specs:
            if name.endswith("layer_norm.weight") or name.endswith("image_pre_norm_module.weight") or \
                    re.search(r"\.(norm[123]|layer_norm1)\.weight$", name):
                t = torch.ones(shape)
            elif name.endswith(".bias") and ("layer_norm" in name or "out_proj" in name or "image_pre_norm" in name
                                             or re.search(r"\.norm[123]\.bias$", name) or "in_proj_bias" in name):
                t = torch.zeros(shape)
            elif name.endswith("embed_tokens.weight"):
                t = torch.randn(shape, generator=g) * shape[1] ** -0.5
                t[self.cfg["padding_idx"]] = 0
            elif len(shape) >= 2:
                fan_out, fan_in = shape[0], int(np.prod(shape[1:]))
                if any(s in name for s in ("q_proj", "k_proj", "v_proj", "in_proj", "out_proj", "gate_denses")):
                    gain = 1 / math.sqrt(2) if "out_proj" not in name and "gate" not in name else 1.0
                    a = gain * math.sqrt(6.0 / (fan_in + fan_out))
                else:
                    a = 1.0 / math.sqrt(fan_in)
                t = (torch.rand(shape, generator=g) * 2 - 1) * a
            elif name.endswith("bias_k") or name.endswith("bias_v"):
                t = torch.randn(shape, generator=g) * math.sqrt(2.0 / (1 + shape[-1]))
            else:
                t = (torch.rand(shape, generator=g) * 2 - 1) * 0.02
            sd[name] = t
        for name, t in self.params.unused.items():
            sd[name] = (torch.rand(t.shape, generator=g) * 2 - 1) * 0.02
        self.params.load_state_dict(sd)
        return self

    def train(self, mode=True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    # -------------------------------------------------------------- helpers
    grad_ready_hook = None  # callable(offset): grads [0, offset) of the flat buffer are final
    grad_release_finish = None  # callable(): after the backward joined its side stream (fairseq_adapter)

    def _ready(self, last_param=None):
        if self.grad_ready_hook is None:
            return
        K.wgrad_flush()   # a deferred weight-gradient group belongs to the gradients reported ready
        if last_param is None:
            self.grad_ready_hook(self.params.numel)
        else:
            off, _, n = self.params.offsets[last_param]
            self.grad_ready_hook(off + n)

    def cross_kv(self, grad=False, spec=None):
        """(W [L_d*2d, de], b [L_d*2d]) of all decoder layers' cross-attention K/V projections."""
        spec = spec or self.dspec
        L = spec.L
        f, t = f"{spec.prefix}.layers.0.encoder_attn", f"{spec.prefix}.layers.{L - 1}.encoder_attn"
        W = self.params.span(f + ".k_proj.weight", t + ".v_proj.weight", grad=grad)
        b = self.params.span(f + ".k_proj.bias", t + ".v_proj.bias", grad=grad)
        return W.view(b.numel(), -1), b

    def P(self, n):
        return self.params.p[n]

    def _zero_grads(self, prefixes):
        """Zero the gradients of every parameter whose name starts with one of `prefixes`: a branch
        whose backward does not run leaves them untouched this step, and nothing else clears the
        gradient buffer (every other gradient is written outright by its backward, see
        ParamStore)."""
        for n, _ in self.params.specs:
            if n.startswith(prefixes):
                self.params.g[n].zero_()

    def G(self, n):
        return self.params.g[n]

    def _p(self, key):
        return self.cfg[key] if self.training else 0.0

    def _drop(self, p, n):
        return self.drop.take(n) if p > 0 else None

    def _ensure_pos(self, T, which):
        if isinstance(which, int):       # a decoder width other than the unit decoder's
            tab = self._pos.get(which)
            if tab is None or T + 2 > tab.shape[0]:
                if tab is not None and self.retain_tables:
                    self._retired.append(tab)
                tab = sinusoidal_table(max(T + 2, 1026), which).to(self.device, F16)
                self._pos[which] = tab
            return tab
        tab = self.enc_pos if which == "enc" else self.dec_pos
        if T + 2 > tab.shape[0]:
            if self.retain_tables:
                self._retired.append(tab)
            dim = tab.shape[1]
            tab = sinusoidal_table(T + 2, dim).to(self.device, F16)
            if which == "enc":
                self.enc_pos = tab
            else:
                self.dec_pos = tab
        return tab

    # -------------------------------------------------------------- subsampler
    def _conv_call(self):
        """The K.ConvCall of the subsampler (bound to its weight / gradient / W^T slots)."""
        if self._conv is None:
            ks = list(self.cfg["conv_kernel_sizes"])
            Ws = [self.P(f"encoder.subsample.conv_layers.{i}.weight") for i in range(len(ks))]
            self._conv = K.ConvCall(
                ks, [W.shape[0] for W in Ws], Ws, [self.P(f"encoder.subsample.conv_layers.{i}.bias") for i in range(len(ks))],
                [self.G(f"encoder.subsample.conv_layers.{i}.weight") for i in range(len(ks))],
                [self.G(f"encoder.subsample.conv_layers.{i}.bias") for i in range(len(ks))],
                {i: Ws[i].view(Ws[i].shape[0], -1) for i in range(1, len(ks))})
        return self._conv

    def subsample_fwd(self, src, lens):
        """fairseq Conv1dSubsampler (conv(k, s2, p k//2) -> GLU per layer) in one library call
        (mms2ut_conv1d_glu_fwd); bit-identical to subsample_fwd_ref."""
        B, Ts, Cin = src.shape
        cc = self._conv_call()
        arena, out, snap = cc.fwd(src.reshape(B * Ts, Cin), B, Ts, Cin)
        return out, out.shape[0] // B, {"arena": arena, "snap": snap}

    def subsample_bwd(self, ctx, dx):
        self._conv_call().bwd(ctx["snap"], ctx["arena"], dx.contiguous())

    def subsample_fwd_ref(self, src, lens):
        """fairseq Conv1dSubsampler: conv(k, s2, p k//2) -> GLU, twice; implicit GEMM, one launch
        at a time from Python (the reference sequence the one-call path is checked against)."""
        cfg = self.cfg
        B, Ts, Cin = src.shape
        ctx = {"B": B, "Ts": Ts, "layers": []}
        x = src.reshape(B * Ts, Cin)
        Tin, C = Ts, Cin
        for i, k in enumerate(cfg["conv_kernel_sizes"]):
            W = self.P(f"encoder.subsample.conv_layers.{i}.weight")
            bias = self.P(f"encoder.subsample.conv_layers.{i}.bias")
            Tout = (Tin - 1) // 2 + 1
            W2 = W.view(W.shape[0], -1)
            ck = C * k
            if ck % 64:
                # K = C*k padded to whole 64-wide k-tiles (zero columns in col and in a padded copy
                # of W) so the projection runs on the LDS-DMA GEMM instead of the predicated one
                kp = -(-ck // 64) * 64
                col = K.im2col(x, B, Tin, Tout, C, k, ldcol=kp)
                Wp = self._wpad.get(i)
                if Wp is None or Wp.shape != (W2.shape[0], kp):
                    Wp = torch.zeros(W2.shape[0], kp, dtype=F16, device=W.device)
                    self._wpad[i] = Wp
                K.copy2d(W2, Wp, W2.shape[0], ck)
                y = K.linear(col, Wp, bias)
                col = col[:, :ck]
            else:
                col = K.im2col(x, B, Tin, Tout, C, k)
                y = K.linear(col, W2, bias)
            Cg = W.shape[0] // 2
            g = K.glu(y, Cg)
            ctx["layers"].append(dict(col=col, y=y, Tin=Tin, Tout=Tout, C=C, k=k, Cg=Cg))
            x, Tin, C = g, Tout, Cg
        return x, Tin, ctx

    def subsample_bwd_ref(self, ctx, dx):
        B = ctx["B"]
        for i in reversed(range(len(ctx["layers"]))):
            L = ctx["layers"][i]
            W = self.P(f"encoder.subsample.conv_layers.{i}.weight")
            dy = K.glu_bwd(L["y"], dx, L["Cg"])
            K.linear_wgrad(dy, L["col"], self.G(f"encoder.subsample.conv_layers.{i}.weight").view(W.shape[0], -1),
                           db=self.G(f"encoder.subsample.conv_layers.{i}.bias"))
            if i > 0:
                dcol = K.linear_dgrad(dy, W.view(W.shape[0], -1))
                dx = K.col2im(dcol, B, L["Tin"], L["Tout"], L["C"], L["k"])

    # -------------------------------------------------------------- transformer layers (one call each)
    def _layer_call(self, prefix, kind, d, H, F):
        """The K.LayerCall of layer ``prefix`` (bound to its parameter / gradient / W^T slots)."""
        lc = self._layer_calls.get(prefix)
        if lc is not None:
            return lc
        P, G, span = self.P, self.G, self.params.span
        q0, v0 = prefix + ".self_attn.q_proj", prefix + ".self_attn.v_proj"
        params = {"ln1_g": P(prefix + ".self_attn_layer_norm.weight"), "ln1_b": P(prefix + ".self_attn_layer_norm.bias"),
                  "w_qkv": span(q0 + ".weight", v0 + ".weight"), "b_qkv": span(q0 + ".bias", v0 + ".bias"),
                  "w_o": P(prefix + ".self_attn.out_proj.weight"), "b_o": P(prefix + ".self_attn.out_proj.bias"),
                  "ln3_g": P(prefix + ".final_layer_norm.weight"), "ln3_b": P(prefix + ".final_layer_norm.bias"),
                  "w_fc1": P(prefix + ".fc1.weight"), "b_fc1": P(prefix + ".fc1.bias"),
                  "w_fc2": P(prefix + ".fc2.weight"), "b_fc2": P(prefix + ".fc2.bias")}
        lns = lambda n: span(n + ".weight", n + ".bias", grad=True)  # noqa: E731
        grads = {"g_ln1": lns(prefix + ".self_attn_layer_norm"), "g_w_qkv": span(q0 + ".weight", v0 + ".weight", grad=True),
                 "g_b_qkv": span(q0 + ".bias", v0 + ".bias", grad=True),
                 "g_w_o": G(prefix + ".self_attn.out_proj.weight"), "g_b_o": G(prefix + ".self_attn.out_proj.bias"),
                 "g_ln3": lns(prefix + ".final_layer_norm"), "g_w_fc1": G(prefix + ".fc1.weight"),
                 "g_b_fc1": G(prefix + ".fc1.bias"), "g_w_fc2": G(prefix + ".fc2.weight"), "g_b_fc2": G(prefix + ".fc2.bias")}
        wts = {"wt_qkv": span(q0 + ".weight", v0 + ".weight").view(3 * d, d), "wt_o": P(prefix + ".self_attn.out_proj.weight"),
               "wt_fc1": P(prefix + ".fc1.weight"), "wt_fc2": P(prefix + ".fc2.weight")}
        if kind == K._lib.LAYER_DEC:
            e = prefix + ".encoder_attn"
            params.update(ln2_g=P(prefix + ".encoder_attn_layer_norm.weight"), ln2_b=P(prefix + ".encoder_attn_layer_norm.bias"),
                          w_cq=P(e + ".q_proj.weight"), b_cq=P(e + ".q_proj.bias"),
                          w_co=P(e + ".out_proj.weight"), b_co=P(e + ".out_proj.bias"))
            grads.update(g_ln2=lns(prefix + ".encoder_attn_layer_norm"), g_w_cq=G(e + ".q_proj.weight"),
                         g_b_cq=G(e + ".q_proj.bias"), g_w_co=G(e + ".out_proj.weight"), g_b_co=G(e + ".out_proj.bias"))
            wts.update(wt_cq=P(e + ".q_proj.weight"), wt_co=P(e + ".out_proj.weight"))
        lc = K.LayerCall(kind, d, H, F, params, grads, wts)
        self._layer_calls[prefix] = lc
        return lc

    def enc_layer_fwd(self, l, x, B, T, lens32):
        """fairseq TransformerEncoderLayer (pre-LN) forward as one library call (mms2ut_layer_fwd).
        Dropout sites draw their counters in the per-launch order (attention, out_proj residual,
        activation, fc2 residual), so masks are those of enc_layer_fwd_ref."""
        cfg = self.cfg
        d, H, F_ = cfg["encoder_embed_dim"], cfg["encoder_attention_heads"], cfg["encoder_ffn_embed_dim"]
        R = B * T
        pd, pa, pact = self._p("dropout"), self._p("attention_dropout"), self._p("activation_dropout")
        c = {"x": x, "B": B, "T": T, "lens32": lens32, "pd": pd, "pa": pa, "pact": pact}
        c["drop_attn"] = self._drop(pa, B * H * T * T)
        c["drop1"] = self._drop(pd, R * d)
        c["drop_act"] = self._drop(pact, R * F_)
        c["drop2"] = self._drop(pd, R * d)
        o = lambda dr: dr[1] if dr else 0  # noqa: E731
        lc = self._layer_call(f"encoder.transformer_layers.{l}", K._lib.LAYER_ENC, d, H, F_)
        arena, offs, snap = lc.fwd(x, B, T, lens32, self.drop.seed, (pd, pa, pact),
                                   (o(c["drop_attn"]), o(c["drop1"]), 0, 0, o(c["drop_act"]), o(c["drop2"])))
        c.update(lc=lc, arena=arena, snap=snap)
        c["f1"] = K.LayerCall.view(arena, offs, K._lib.SLOT_F1, (R, F_))
        return K.LayerCall.view(arena, offs, K._lib.SLOT_OUT, (R, d)), c

    def enc_layer_bwd(self, l, c, dx3, dy2=None, emit=None):
        """Backward of enc_layer_fwd (mms2ut_layer_bwd): dx3 = gradient of the layer output, dy2 =
        dropout(dx3) with the fc2-residual mask when the layer above produced it, emit = (p, drop)
        of the layer below's fc2 residual.  Returns (dx, masked dx or None)."""
        dx, dxd = c["lc"].bwd(c["snap"], c["arena"], dx3, c["B"] * c["T"], dy_drop=dy2, emit=emit, last=l == 0)
        return dx, (dxd if emit is not None else None)

    def dec_layer_fwd(self, l, x, kv_all, B, Tt, Te, tgt_mask, enc_len32, tgt_len32=None, spec=None):
        """fairseq TransformerDecoderLayer (pre-LN) forward as one library call; the cross-attention
        K | V are this layer's columns of the batched projection kv_all."""
        spec = spec or self.dspec
        if tgt_len32 is None:
            raise NotImplementedError("decoder layers need right-padded targets (fairseq collate_tokens, left_pad=False)")
        p = f"{spec.prefix}.layers.{l}"
        d, H, F_ = spec.d, spec.H, spec.F
        R = B * Tt
        pd, pa, pact = self._sp(spec.pd), self._sp(spec.pa), self._sp(spec.pact)
        c = {"x": x, "B": B, "Tt": Tt, "Te": Te, "pd": pd, "pa": pa, "pact": pact}
        c["drop_sa"] = self._drop(pa, B * H * Tt * Tt)
        c["drop1"] = self._drop(pd, R * d)
        c["drop_ca"] = self._drop(pa, B * H * Tt * Te)
        c["drop2"] = self._drop(pd, R * d)
        c["drop_act"] = self._drop(pact, R * F_)
        c["drop3"] = self._drop(pd, R * d)
        o = lambda dr: dr[1] if dr else 0  # noqa: E731
        lc = self._layer_call(p, K._lib.LAYER_DEC, d, H, F_)
        kv = kv_all[:, 2 * d * l:2 * d * (l + 1)]
        arena, offs, snap = lc.fwd(x, B, Tt, tgt_len32, self.drop.seed, (pd, pa, pact),
                                   (o(c["drop_sa"]), o(c["drop1"]), o(c["drop_ca"]), o(c["drop2"]), o(c["drop_act"]),
                                    o(c["drop3"])), Tk=Te, cross_len=enc_len32, kv=kv)
        c.update(lc=lc, arena=arena, snap=snap)
        c["f1"] = K.LayerCall.view(arena, offs, K._lib.SLOT_F1, (R, F_))
        return K.LayerCall.view(arena, offs, K._lib.SLOT_OUT, (R, d)), c

    def dec_layer_bwd(self, l, c, dx4, dkv_all, dy3=None, emit=None, spec=None):
        """Backward of dec_layer_fwd; writes this layer's K | V gradient into its dkv_all columns."""
        spec = spec or self.dspec
        d = spec.d
        dkv = dkv_all[:, 2 * d * l:2 * d * (l + 1)]
        dx, dxd = c["lc"].bwd(c["snap"], c["arena"], dx4, c["B"] * c["Tt"], dy_drop=dy3, emit=emit, dkv=dkv)
        return dx, (dxd if emit is not None else None)

    # -------------------------------------------------------------- encoder layer (per-launch reference)
    def enc_layer_fwd_ref(self, l, x, B, T, lens32):
        cfg = self.cfg
        p = f"encoder.transformer_layers.{l}"
        d, H = cfg["encoder_embed_dim"], cfg["encoder_attention_heads"]
        hd = d // H
        R = B * T
        c = {"x": x}
        h1, c["m1"], c["r1"] = K.layernorm(x, self.P(p + ".self_attn_layer_norm.weight"),
                                           self.P(p + ".self_attn_layer_norm.bias"))
        c["h1"] = h1
        Wqkv = self.params.span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight").view(3 * d, d)
        bqkv = self.params.span(p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias")
        qkv = K.linear(h1, Wqkv, bqkv)
        c["qkv"] = qkv
        O = torch.empty(R, d, dtype=F16, device=x.device)
        pa = self._p("attention_dropout")
        c["drop_attn"] = self._drop(pa, B * H * T * T)
        c["attn"] = attn_forward(qkv, qkv[:, d:], qkv[:, 2 * d:], 3 * d, 3 * d, 3 * d, B, H, T, T, hd,
                                 hd ** -0.5, O, d, key_len=lens32, p=pa, drop=c["drop_attn"])
        c["O"] = O
        pd = self._p("dropout")
        c["drop1"] = self._drop(pd, R * d)
        x2 = K.linear(O, self.P(p + ".self_attn.out_proj.weight"), self.P(p + ".self_attn.out_proj.bias"),
                      epi=K.EPI_DROP_RESID, aux=x, p=pd, drop=c["drop1"])
        c["x2"] = x2
        h2, c["m2"], c["r2"] = K.layernorm(x2, self.P(p + ".final_layer_norm.weight"),
                                           self.P(p + ".final_layer_norm.bias"))
        c["h2"] = h2
        pact = self._p("activation_dropout")
        c["drop_act"] = self._drop(pact, R * cfg["encoder_ffn_embed_dim"])
        F_ = cfg["encoder_ffn_embed_dim"]
        f1 = K.linear(h2, self.P(p + ".fc1.weight"), self.P(p + ".fc1.bias"), epi=K.EPI_RELU_DROP,
                      p=pact, drop=c["drop_act"])
        c["f1"] = f1
        c["drop2"] = self._drop(pd, R * d)
        x3 = K.linear(f1, self.P(p + ".fc2.weight"), self.P(p + ".fc2.bias"), epi=K.EPI_DROP_RESID,
                      aux=x2, p=pd, drop=c["drop2"])
        c.update(B=B, T=T, lens32=lens32, pd=pd, pa=pa, pact=pact)
        return x3, c

    def enc_layer_bwd_ref(self, l, c, dx3, dy2=None, emit=None):
        """dx3: gradient of the layer output; dy2: dropout(dx3) with this layer's fc2-branch mask
        when the LayerNorm backward above already produced it.  emit=(p, drop) makes this
        layer's first LayerNorm backward also produce the masked gradient for the layer below.
        Returns (dx, dx masked by emit or None)."""
        cfg = self.cfg
        p = f"encoder.transformer_layers.{l}"
        d, H = cfg["encoder_embed_dim"], cfg["encoder_attention_heads"]
        hd = d // H
        B, T = c["B"], c["T"]
        pd, pa, pact = c["pd"], c["pa"], c["pact"]
        # fc2 / fc1
        if dy2 is None:
            dy2 = K.dropout(dx3, pd, c["drop2"], out=torch.empty_like(dx3)) if pd > 0 else dx3
        # the critical-path dgrad is enqueued before the side-stream weight gradient that reads
        # the same dy, so its blocks are dispatched first
        df1 = K.linear_dgrad(dy2, self.P(p + ".fc2.weight"), epi=K.EPI_RELU_DROP_BWD, aux=c["f1"], p=pact)
        K.linear_wgrad(dy2, c["f1"], self.G(p + ".fc2.weight"), db=self.G(p + ".fc2.bias"))
        dh2 = K.linear_dgrad(df1, self.P(p + ".fc1.weight"))
        K.linear_wgrad(df1, c["h2"], self.G(p + ".fc1.weight"), db=self.G(p + ".fc1.bias"))
        del df1
        dx2, dyo = K.layernorm_bwd(dh2, c["x2"], self.P(p + ".final_layer_norm.weight"), c["m2"], c["r2"],
                                   self.params.span(p + ".final_layer_norm.weight", p + ".final_layer_norm.bias", grad=True),
                                   dres=dx3, emit=(pd, c["drop1"]))
        # out proj (dyo = dropout(dx2) with the attention-branch mask, from the LN backward)
        dO = K.linear_dgrad(dyo, self.P(p + ".self_attn.out_proj.weight"))
        K.linear_wgrad(dyo, c["O"], self.G(p + ".self_attn.out_proj.weight"),
                       db=self.G(p + ".self_attn.out_proj.bias"))
        qkv = c["qkv"]
        dqkv = torch.empty_like(qkv)
        attn_backward(c["attn"], dO, d, c["O"], qkv, qkv[:, d:], qkv[:, 2 * d:], 3 * d, 3 * d, 3 * d,
                      B, H, T, T, hd, hd ** -0.5, dqkv, dqkv[:, d:], dqkv[:, 2 * d:], 3 * d, 3 * d, 3 * d,
                      p=pa, drop=c["drop_attn"])
        Wqkv = self.params.span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight").view(3 * d, d)

        def qkv_wgrad():
            K.linear_wgrad(dqkv, c["h1"], self.params.span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight", grad=True).view(3 * d, d),
                           db=self.params.span(p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias", grad=True))
        dh1 = K.linear_dgrad(dqkv, Wqkv)
        qkv_wgrad()
        if emit is None:
            dx = K.layernorm_bwd(dh1, c["x"], self.P(p + ".self_attn_layer_norm.weight"), c["m1"], c["r1"],
                                 self.params.span(p + ".self_attn_layer_norm.weight", p + ".self_attn_layer_norm.bias", grad=True),
                                 dres=dx2)
            return dx, None
        return K.layernorm_bwd(dh1, c["x"], self.P(p + ".self_attn_layer_norm.weight"), c["m1"], c["r1"],
                               self.params.span(p + ".self_attn_layer_norm.weight", p + ".self_attn_layer_norm.bias", grad=True),
                               dres=dx2, emit=emit)

    # -------------------------------------------------------------- fusion (fuse_img_feat)
    def _fusion_call(self, Di):
        """The K.FusionCall of the fusion tail (bound to its parameter / gradient / W^T slots)."""
        fc = self._fusion.get(Di)
        if fc is not None:
            return fc
        cfg, P, G, span = self.cfg, self.P, self.G, self.params.span
        d = cfg["encoder_embed_dim"]
        extra = cfg["multimodal_attention_type"] == "multimodal_attention"
        if extra:
            pre = "encoder.multimodal_attns.0"
            if Di == d:
                W, gW = P(pre + ".in_proj_weight"), G(pre + ".in_proj_weight")
                Wq, Wkv, gWq, gWkv = W[:d], W[d:], gW[:d], gW[d:]
            else:
                Wq, gWq = P(pre + ".q_proj_weight"), G(pre + ".q_proj_weight")
                Wkv = span(pre + ".k_proj_weight", pre + ".v_proj_weight").view(2 * d, Di)
                gWkv = span(pre + ".k_proj_weight", pre + ".v_proj_weight", grad=True).view(2 * d, Di)
            b, gb = P(pre + ".in_proj_bias"), G(pre + ".in_proj_bias")
            bq, bkv, gbq, gbkv = b[:d], b[d:], gb[:d], gb[d:]
            Wo, bo, gWo, gbo = (P(pre + ".out_proj.weight"), P(pre + ".out_proj.bias"), G(pre + ".out_proj.weight"),
                                G(pre + ".out_proj.bias"))
            bias_kv, g_bias_kv = span(pre + ".bias_k", pre + ".bias_v"), span(pre + ".bias_k", pre + ".bias_v", grad=True)
        else:
            pre = "encoder.selective_attns.0"
            Wq, bq, gWq, gbq = (P(pre + ".q_proj.weight"), P(pre + ".q_proj.bias"), G(pre + ".q_proj.weight"),
                                G(pre + ".q_proj.bias"))
            Wkv = span(pre + ".k_proj.weight", pre + ".v_proj.weight").view(2 * d, Di)
            gWkv = span(pre + ".k_proj.weight", pre + ".v_proj.weight", grad=True).view(2 * d, Di)
            bkv, gbkv = span(pre + ".k_proj.bias", pre + ".v_proj.bias"), span(pre + ".k_proj.bias", pre + ".v_proj.bias", grad=True)
            Wo, bo, gWo, gbo = P(pre + ".proj.weight"), P(pre + ".proj.bias"), G(pre + ".proj.weight"), G(pre + ".proj.bias")
            bias_kv = g_bias_kv = None
        gate, pre_norm = bool(cfg["use_selective_gate"]), bool(cfg["image_pre_norm"])
        ln = "encoder.image_pre_norm_module"
        params = {"ln_g": P(ln + ".weight") if pre_norm else None, "ln_b": P(ln + ".bias") if pre_norm else None,
                  "wq": Wq, "bq": bq, "wkv": Wkv, "bkv": bkv, "bias_kv": bias_kv, "wo": Wo, "bo": bo,
                  "wg": P("encoder.gate_denses.0.weight") if gate else None,
                  "bg": P("encoder.gate_denses.0.bias") if gate else None}
        grads = {"g_ln": span(ln + ".weight", ln + ".bias", grad=True) if pre_norm else None,
                 "g_wq": gWq, "g_bq": gbq, "g_wkv": gWkv, "g_bkv": gbkv, "g_bias_kv": g_bias_kv, "g_wo": gWo, "g_bo": gbo,
                 "g_wg": G("encoder.gate_denses.0.weight") if gate else None,
                 "g_bg": G("encoder.gate_denses.0.bias") if gate else None}
        wts = {"wt_q": Wq, "wt_kv": Wkv, "wt_o": Wo}
        if gate:
            wts["wt_g"] = P("encoder.gate_denses.0.weight")
        flags = {"d": d, "Di": Di, "extra": int(extra), "gate": int(gate), "image_pre_norm": int(pre_norm), "eps": 1e-5}
        fc = K.FusionCall(flags, params, grads, wts)
        self._fusion[Di] = fc
        return fc

    def fusion_fwd(self, text, img, img_mask, B, Te):
        """mm_s2s_transformer.py:594-622 in one library call (mms2ut_gated_fusion_fwd); the same
        dropout draws and bit-identical results as fusion_fwd_ref.  text [B*Te, d] (encoder out),
        img [B, Ti, Di] fp16."""
        cfg = self.cfg
        d = cfg["encoder_embed_dim"]
        _, Ti, Di = img.shape
        extra = cfg["multimodal_attention_type"] == "multimodal_attention"
        Tk = Ti + 1 if extra else Ti
        pimg, ptxt, pat = self._p("SA_image_dropout"), self._p("SA_text_dropout"), self._p("SA_attention_dropout")
        drops = (self._drop(pimg, B * Ti * Di), self._drop(ptxt, B * Te * d), self._drop(pat, B * Te * Tk))
        img2 = img.reshape(B * Ti, Di).contiguous()
        text = text.contiguous()
        arena, out, snap = self._fusion_call(Di).fwd(text, img2, img_mask, B, Te, Ti, (pimg, ptxt, pat), drops)
        c = {"B": B, "Te": Te, "Ti": Ti, "Di": Di, "Tk": Tk, "extra": extra, "pimg": pimg, "ptxt": ptxt, "pat": pat,
             "drop_img": drops[0], "drop_txt": drops[1], "drop_attn": drops[2], "arena": arena, "snap": snap,
             "keep": tuple(t for t in (text, img2, img_mask) if t is not None)}
        return out, c

    def fusion_bwd(self, c, dres, want_dimg=False):
        """-> d(text) [B*Te, d]; with want_dimg also d(img) [B*Ti, Di] (mms2ut_gated_fusion_bwd)."""
        return self._fusion_call(c["Di"]).bwd(c["snap"], c["arena"], c["keep"], dres.contiguous(), want_dimg)

    def fusion_fwd_ref(self, text, img, img_mask, B, Te):
        """mm_s2s_transformer.py:594-622, one launch at a time from Python (the reference sequence
        the one-call path is checked against). text [B*Te, d] (encoder out), img [B, Ti, Di] fp16."""
        cfg = self.cfg
        d = cfg["encoder_embed_dim"]
        _, Ti, Di = img.shape
        att = cfg["multimodal_attention_type"]
        extra = att == "multimodal_attention"  # add_bias_kv: one learned key/value row
        Tk = Ti + 1 if extra else Ti
        c = {"B": B, "Te": Te, "Ti": Ti, "Di": Di, "Tk": Tk, "extra": extra}
        # image_pre_norm (+ dropout), laid out [B, Tk, Di] with a zero row per batch for bias_kv
        img2 = img.reshape(B * Ti, Di)
        pimg = self._p("SA_image_dropout")
        c["drop_img"] = self._drop(pimg, B * Ti * Di)
        c["ln_fused"] = cfg["image_pre_norm"] and Di % 256 == 0 and Di <= 1024
        if c["ln_fused"]:
            # LN -> dropout -> [B, Tk, Di] key layout in one pass (layernorm_fwd_ex); the extra
            # bias_kv row per batch is zeroed separately
            imgd = torch.empty(B, Tk, Di, dtype=F16, device=img.device)
            if extra:
                imgd[:, Ti:].zero_()
            _, c["im"], c["ir"] = K.layernorm(img2, self.P("encoder.image_pre_norm_module.weight"),
                                              self.P("encoder.image_pre_norm_module.bias"), out=imgd,
                                              grp=Ti if extra else 0, grp_out=Tk if extra else 0, p=pimg,
                                              drop=c["drop_img"])
            c["img_in"] = img2
            imgd = imgd.view(B * Tk, Di)
        else:
            if cfg["image_pre_norm"]:
                imgn, c["im"], c["ir"] = K.layernorm(img2, self.P("encoder.image_pre_norm_module.weight"),
                                                     self.P("encoder.image_pre_norm_module.bias"))
                c["img_in"] = img2
            else:
                imgn = img2
            if pimg > 0:
                imgn = K.dropout(imgn, pimg, c["drop_img"])
            if extra:
                imgd = torch.zeros(B, Tk, Di, dtype=F16, device=img.device)
                K.copy2d(imgn.view(B, Ti * Di), imgd.view(B, Tk * Di), B, Ti * Di)
                imgd = imgd.view(B * Tk, Di)
            else:
                imgd = imgn
        c["imgd"] = imgd
        ptxt = self._p("SA_text_dropout")
        c["drop_txt"] = self._drop(ptxt, B * Te * d)
        textd = K.dropout(text, ptxt, c["drop_txt"], out=torch.empty_like(text)) if ptxt > 0 else text
        c["textd"] = textd
        if extra:
            pre = "encoder.multimodal_attns.0"
            if Di == d:
                W = self.P(pre + ".in_proj_weight")
                Wq, Wkv = W[:d], W[d:]
            else:
                Wq = self.P(pre + ".q_proj_weight")
                Wkv = self.params.span(pre + ".k_proj_weight", pre + ".v_proj_weight").view(2 * d, Di)
            bias = self.P(pre + ".in_proj_bias")
            bq, bkv = bias[:d], bias[d:]
            Wo, bo = self.P(pre + ".out_proj.weight"), self.P(pre + ".out_proj.bias")
        else:
            pre = "encoder.selective_attns.0"
            Wq, bq = self.P(pre + ".q_proj.weight"), self.P(pre + ".q_proj.bias")
            Wkv = self.params.span(pre + ".k_proj.weight", pre + ".v_proj.weight").view(2 * d, Di)
            bkv = self.params.span(pre + ".k_proj.bias", pre + ".v_proj.bias")
            Wo, bo = self.P(pre + ".proj.weight"), self.P(pre + ".proj.bias")
        c["pre"] = pre
        q = K.linear(textd, Wq, bq)
        kv = K.linear(imgd, Wkv, bkv)                      # [B*Tk, 2d]
        if extra:
            bkv_rows = self.params.span(pre + ".bias_k", pre + ".bias_v").view(1, 2 * d)
            K.copy2d(bkv_rows.expand(B, 2 * d), kv.view(B, Tk * 2 * d)[:, Ti * 2 * d:], B, 2 * d)
        c["q"], c["kv"] = q, kv
        key_mask = img_mask  # uint8 [B, >=Tk] prepared by prepare_batch (1 = padded key)
        c["key_mask"] = key_mask
        pat = self._p("SA_attention_dropout")
        c["drop_attn"] = self._drop(pat, B * Te * Tk)
        O = torch.empty(B * Te, d, dtype=F16, device=text.device)
        c["P"], c["Pd"], c["ldS"] = attn_fwd(q, kv, kv[:, d:], d, 2 * d, 2 * d, B, 1, Te, Tk, d,
                                             d ** -0.5, O, d, key_mask=key_mask, extra_key=extra,
                                             p=pat, drop=c["drop_attn"])
        c["O"], c["pat"], c["pimg"], c["ptxt"] = O, pat, pimg, ptxt
        if cfg["use_selective_gate"]:
            merge = torch.empty(B * Te, 2 * d, dtype=F16, device=text.device)
            K.linear(O, Wo, bo, out=merge[:, :d], ldc=2 * d)
            K.copy2d(textd, merge[:, d:], B * Te, d)
            g = torch.empty(B * Te, d, dtype=F16, device=text.device)
            res = K.linear(merge, self.P("encoder.gate_denses.0.weight"), self.P("encoder.gate_denses.0.bias"),
                           epi=K.EPI_GATE, aux=merge, out2=g)
            c["merge"], c["g"] = merge, g
        else:
            res = K.linear(O, Wo, bo, epi=K.EPI_DROP_RESID, aux=textd)
        return res, c

    def fusion_bwd_ref(self, c, dres, want_dimg=False):
        """-> d(text) [B*Te, d]; with want_dimg also d(img) [B*Ti, Di] (the image features are not
        leaves behind a QFormer)."""
        cfg = self.cfg
        d = cfg["encoder_embed_dim"]
        B, Te, Ti, Di, Tk, extra, pre = c["B"], c["Te"], c["Ti"], c["Di"], c["Tk"], c["extra"], c["pre"]
        if extra:
            if Di == d:
                W = self.P(pre + ".in_proj_weight")
                Wq, Wkv = W[:d], W[d:]
                gW = self.G(pre + ".in_proj_weight")
                gWq, gWkv = gW[:d], gW[d:]
            else:
                Wq = self.P(pre + ".q_proj_weight")
                Wkv = self.params.span(pre + ".k_proj_weight", pre + ".v_proj_weight").view(2 * d, Di)
                gWq = self.G(pre + ".q_proj_weight")
                gWkv = self.params.span(pre + ".k_proj_weight", pre + ".v_proj_weight", grad=True).view(2 * d, Di)
            gb = self.G(pre + ".in_proj_bias")
            gbq, gbkv = gb[:d], gb[d:]
            Wo, gWo, gbo = self.P(pre + ".out_proj.weight"), self.G(pre + ".out_proj.weight"), self.G(pre + ".out_proj.bias")
        else:
            Wq, gWq, gbq = self.P(pre + ".q_proj.weight"), self.G(pre + ".q_proj.weight"), self.G(pre + ".q_proj.bias")
            Wkv = self.params.span(pre + ".k_proj.weight", pre + ".v_proj.weight").view(2 * d, Di)
            gWkv = self.params.span(pre + ".k_proj.weight", pre + ".v_proj.weight", grad=True).view(2 * d, Di)
            gbkv = self.params.span(pre + ".k_proj.bias", pre + ".v_proj.bias", grad=True)
            Wo, gWo, gbo = self.P(pre + ".proj.weight"), self.G(pre + ".proj.weight"), self.G(pre + ".proj.bias")
        if cfg["use_selective_gate"]:
            dpre, dmerge = K.gate_bwd(dres, c["merge"], c["g"])
            K.linear_wgrad(dpre, c["merge"], self.G("encoder.gate_denses.0.weight"),
                           db=self.G("encoder.gate_denses.0.bias"))
            K.linear_dgrad(dpre, self.P("encoder.gate_denses.0.weight"), out=dmerge, accumulate=True)
            dOp = dmerge[:, :d]
            dtext = dmerge[:, d:]
        else:
            dOp = dres
            dtext = dres
        K.linear_wgrad(dOp, c["O"], gWo,
                       db=gbo)
        dO = K.linear_dgrad(dOp, Wo)
        q, kv = c["q"], c["kv"]
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        attn_bwd(dO, d, q, kv, kv[:, d:], d, 2 * d, 2 * d, c["P"], c["Pd"], c["ldS"], B, 1, Te, Tk, d,
                 d ** -0.5, dq, dkv, dkv[:, d:], d, 2 * d, 2 * d, p=c["pat"], drop=c["drop_attn"])
        if extra:
            # bias_k / bias_v grads = sum over batch of the extra key row; then zero that row
            rows = dkv.view(B, Tk * 2 * d)[:, Ti * 2 * d:]
            # on the main stream: the rows are zeroed right after (side-stream race otherwise)
            K.bias_grad(rows, self.params.span(pre + ".bias_k", pre + ".bias_v", grad=True), side=False)
            rows.zero_()
        K.linear_wgrad(dkv, c["imgd"], gWkv,
                       db=gbkv)
        dimg_in = None
        if c["ln_fused"]:
            # image LN gamma/beta grads read dimgd through the key layout + dropout directly
            dimgd = K.linear_dgrad(dkv, Wkv)
            dimg_in = K.layernorm_bwd(dimgd, c["img_in"], self.P("encoder.image_pre_norm_module.weight"), c["im"],
                                      c["ir"], self.params.span("encoder.image_pre_norm_module.weight",
                                                                "encoder.image_pre_norm_module.bias", grad=True),
                                      want_dx=want_dimg, dy_grp=Ti if extra else 0, dy_grp_out=Tk if extra else 0,
                                      dy_p=c["pimg"], dy_drop=c["drop_img"])
        elif cfg["image_pre_norm"] or want_dimg:
            dimgd = K.linear_dgrad(dkv, Wkv)
            if extra:
                dimg = torch.empty(B * Ti, Di, dtype=F16, device=dkv.device)
                K.copy2d(dimgd.view(B, Tk * Di), dimg.view(B, Ti * Di), B, Ti * Di)
            else:
                dimg = dimgd
            if c["pimg"] > 0:
                dimg = K.dropout(dimg, c["pimg"], c["drop_img"])
            if cfg["image_pre_norm"]:
                dimg_in = K.layernorm_bwd(dimg, c["img_in"], self.P("encoder.image_pre_norm_module.weight"), c["im"],
                                          c["ir"], self.params.span("encoder.image_pre_norm_module.weight",
                                                                    "encoder.image_pre_norm_module.bias", grad=True),
                                          want_dx=want_dimg)
            else:
                dimg_in = dimg
        K.linear_wgrad(dq, c["textd"], gWq,
                       db=gbq)
        dtext_total = torch.empty(B * Te, d, dtype=F16, device=dres.device)
        K.copy2d(dtext, dtext_total, B * Te, d)
        K.linear_dgrad(dq, Wq, out=dtext_total, accumulate=True)
        if c["ptxt"] > 0:
            dtext_total = K.dropout(dtext_total, c["ptxt"], c["drop_txt"])
        if want_dimg:
            return dtext_total, dimg_in
        return dtext_total

    # -------------------------------------------------------------- post-LN multimodal decoder layers
    def _mha_w(self, p, d, kdim, grad=False):
        """(Wq, Wkv, bq, bkv) of nn.MultiheadAttention `p` (fuse.py:205-209): the packed
        in_proj_weight when kdim == embed_dim, else q/k/v_proj_weight (k and v adjacent)."""
        b = (self.G if grad else self.P)(p + ".in_proj_bias")
        if kdim == d:
            W = (self.G if grad else self.P)(p + ".in_proj_weight")
            return W[:d], W[d:], b[:d], b[d:]
        return ((self.G if grad else self.P)(p + ".q_proj_weight"),
                self.params.span(p + ".k_proj_weight", p + ".v_proj_weight", grad=grad).view(2 * d, kdim), b[:d], b[d:])

    def mml_fwd(self, p, x, mem2, B, Tq, Tm, d, kdim, H, pp, sa_first=True, self_len=None, mem_len=None,
                mem_km=None):
        """MultimodalTransformerDecoderLayer.forward (fuse.py:236-285; norm_first False, GELU):
        self_attention_first: x = norm1(x + drop(SA(x))); x = norm2(x + drop(MHA(x, mem)))
        else:                 x = norm2(x + drop(MHA(x, mem))); x = norm1(x + drop(SA(x)))
        then                  x = norm3(x + drop(linear2(drop(gelu(linear1(x)))))).
        x [B*Tq, d]; mem2 [B*Tm, kdim]; self_len: query lengths (None: every query valid); memory
        keys masked by mem_len (lengths) or mem_km (uint8 key mask)."""
        hd = d // H
        R = B * Tq
        dev = x.device
        c = {"x": x, "pp": pp, "B": B, "Te": Tq, "Ti": Tm, "img2": mem2, "d": d, "kdim": kdim, "H": H, "p": p,
             "sa_first": sa_first}

        def sa_block(xin):
            qkv = K.linear(xin, self.P(p + ".self_attn.in_proj_weight"), self.P(p + ".self_attn.in_proj_bias"))
            O = torch.empty(R, d, dtype=F16, device=dev)
            c["drop_sa"] = self._drop(pp, B * H * Tq * Tq)
            c["sattn"] = attn_forward(qkv, qkv[:, d:], qkv[:, 2 * d:], 3 * d, 3 * d, 3 * d, B, H, Tq, Tq, hd,
                                      hd ** -0.5, O, d, key_len=self_len, p=pp, drop=c["drop_sa"])
            c["qkv"], c["sO"], c["sa_in"] = qkv, O, xin
            c["drop1"] = self._drop(pp, R * d)
            y1 = K.linear(O, self.P(p + ".self_attn.out_proj.weight"), self.P(p + ".self_attn.out_proj.bias"),
                          epi=K.EPI_DROP_RESID, aux=xin, p=pp, drop=c["drop1"])
            x1, c["m1"], c["r1"] = K.layernorm(y1, self.P(p + ".norm1.weight"), self.P(p + ".norm1.bias"))
            c["y1"], c["x1"] = y1, x1
            return x1

        def ca_block(xin):
            Wq, Wkv, bq, bkv = self._mha_w(p + ".multihead_attn", d, kdim)
            q = K.linear(xin, Wq, bq)
            kv = K.linear(mem2, Wkv, bkv)
            O2 = torch.empty(R, d, dtype=F16, device=dev)
            c["drop_ca"] = self._drop(pp, B * H * Tq * Tm)
            c["cattn"] = attn_forward(q, kv, kv[:, d:], d, 2 * d, 2 * d, B, H, Tq, Tm, hd, hd ** -0.5, O2, d,
                                      key_len=mem_len, key_mask=mem_km, p=pp, drop=c["drop_ca"])
            c["q"], c["kv"], c["cO"], c["ca_in"] = q, kv, O2, xin
            c["drop2"] = self._drop(pp, R * d)
            y2 = K.linear(O2, self.P(p + ".multihead_attn.out_proj.weight"), self.P(p + ".multihead_attn.out_proj.bias"),
                          epi=K.EPI_DROP_RESID, aux=xin, p=pp, drop=c["drop2"])
            x2, c["m2"], c["r2"] = K.layernorm(y2, self.P(p + ".norm2.weight"), self.P(p + ".norm2.bias"))
            c["y2"], c["x2"] = y2, x2
            return x2

        xa = ca_block(sa_block(x)) if sa_first else sa_block(ca_block(x))
        F_ = self.P(p + ".linear1.weight").shape[0]
        c["ff_in"] = xa
        c["drop_act"] = self._drop(pp, R * F_)
        z = torch.empty(R, F_, dtype=F16, device=dev)
        h = K.linear(xa, self.P(p + ".linear1.weight"), self.P(p + ".linear1.bias"), epi=K.EPI_GELU_DROP, out2=z,
                     p=pp, drop=c["drop_act"])
        c["z"], c["h"] = z, h
        c["drop3"] = self._drop(pp, R * d)
        y3 = K.linear(h, self.P(p + ".linear2.weight"), self.P(p + ".linear2.bias"), epi=K.EPI_DROP_RESID, aux=xa,
                      p=pp, drop=c["drop3"])
        x3, c["m3"], c["r3"] = K.layernorm(y3, self.P(p + ".norm3.weight"), self.P(p + ".norm3.bias"))
        c["y3"] = y3
        return x3, c

    def _lnspan(self, n):
        return self.params.span(n + ".weight", n + ".bias", grad=True)

    def mml_bwd(self, c, dx3, dmem=None, dmem_accumulate=False):
        """Hand-written backward of mml_fwd: returns d(layer input).  Post-LN: every residual add
        happens before a LayerNorm, so each sublayer's input gradient is (LayerNorm backward) + (the
        sublayer's dgrad), summed into a fresh buffer (the LayerNorm output is still read by
        side-stream weight gradients).  dmem [B*Tm, kdim]: receives the memory's gradient (added to
        its contents with dmem_accumulate); None: the memory is a leaf (image features)."""
        p, d, kdim, H = c["p"], c["d"], c["kdim"], c["H"]
        hd = d // H
        B, Tq, Tm, pp = c["B"], c["Te"], c["Ti"], c["pp"]
        dy3, dl2 = K.layernorm_bwd(dx3, c["y3"], self.P(p + ".norm3.weight"), c["m3"], c["r3"], self._lnspan(p + ".norm3"),
                                   emit=(pp, c["drop3"]))
        dz = K.linear_dgrad(dl2, self.P(p + ".linear2.weight"), epi=K.EPI_GELU_DROP_BWD, aux=c["z"], p=pp,
                            drop=c["drop_act"])
        K.linear_wgrad(dl2, c["h"], self.G(p + ".linear2.weight"), db=self.G(p + ".linear2.bias"))
        dxa = K.add_f16(K.linear_dgrad(dz, self.P(p + ".linear1.weight")), dy3)
        K.linear_wgrad(dz, c["ff_in"], self.G(p + ".linear1.weight"), db=self.G(p + ".linear1.bias"))

        def ca_bwd(dxo):
            dy2, dlo2 = K.layernorm_bwd(dxo, c["y2"], self.P(p + ".norm2.weight"), c["m2"], c["r2"],
                                        self._lnspan(p + ".norm2"), emit=(pp, c["drop2"]))
            dO2 = K.linear_dgrad(dlo2, self.P(p + ".multihead_attn.out_proj.weight"))
            K.linear_wgrad(dlo2, c["cO"], self.G(p + ".multihead_attn.out_proj.weight"),
                           db=self.G(p + ".multihead_attn.out_proj.bias"))
            q, kv = c["q"], c["kv"]
            dq, dkv = torch.empty_like(q), torch.empty_like(kv)
            attn_backward(c["cattn"], dO2, d, c["cO"], q, kv, kv[:, d:], d, 2 * d, 2 * d, B, H, Tq, Tm, hd, hd ** -0.5,
                          dq, dkv, dkv[:, d:], d, 2 * d, 2 * d, p=pp, drop=c["drop_ca"])
            Wq, Wkv, _, _ = self._mha_w(p + ".multihead_attn", d, kdim)
            gWq, gWkv, gbq, gbkv = self._mha_w(p + ".multihead_attn", d, kdim, grad=True)
            dx = K.add_f16(K.linear_dgrad(dq, Wq), dy2)
            K.linear_wgrad(dq, c["ca_in"], gWq, db=gbq)
            K.linear_wgrad(dkv, c["img2"], gWkv, db=gbkv)
            if dmem is not None:
                K.linear_dgrad(dkv, Wkv, out=dmem, accumulate=dmem_accumulate)
            return dx

        def sa_bwd(dxo):
            dy1, dso = K.layernorm_bwd(dxo, c["y1"], self.P(p + ".norm1.weight"), c["m1"], c["r1"],
                                       self._lnspan(p + ".norm1"), emit=(pp, c["drop1"]))
            dO = K.linear_dgrad(dso, self.P(p + ".self_attn.out_proj.weight"))
            K.linear_wgrad(dso, c["sO"], self.G(p + ".self_attn.out_proj.weight"), db=self.G(p + ".self_attn.out_proj.bias"))
            qkv = c["qkv"]
            dqkv = torch.empty_like(qkv)
            attn_backward(c["sattn"], dO, d, c["sO"], qkv, qkv[:, d:], qkv[:, 2 * d:], 3 * d, 3 * d, 3 * d, B, H, Tq, Tq,
                          hd, hd ** -0.5, dqkv, dqkv[:, d:], dqkv[:, 2 * d:], 3 * d, 3 * d, 3 * d, p=pp, drop=c["drop_sa"])
            dx = K.add_f16(K.linear_dgrad(dqkv, self.P(p + ".self_attn.in_proj_weight")), dy1)
            K.linear_wgrad(dqkv, c["sa_in"], self.G(p + ".self_attn.in_proj_weight"),
                           db=self.G(p + ".self_attn.in_proj_bias"))
            return dx

        return sa_bwd(ca_bwd(dxa)) if c["sa_first"] else ca_bwd(sa_bwd(dxa))

    # -------------------------------------------------------------- external multimodal transformer
    def ext_layer_fwd(self, i, x, img2, B, Te, Ti, lens32, img_km):
        """Layer i of ExternalMultimodalTransformerEncoder (fuse.py:298-311: kdim = vdim = Di,
        self-attention first); x [B*Te, d], img2 [B*Ti, Di]."""
        d, Di, H, _, _, _ = external_dims(self.cfg)
        return self.mml_fwd(f"{EXT}.layers.{i}", x, img2, B, Te, Ti, d, Di, H, self._p("SA_attention_dropout"),
                            sa_first=True, self_len=lens32, mem_km=img_km)

    def ext_layer_bwd(self, i, c, dx3):
        return self.mml_bwd(c, dx3)   # the image features are leaves: no memory gradient

    def ext_fwd(self, states, img, img_km, B, Te, lens32):
        """ExternalMultimodalTransformerEncoder.forward (fuse.py:323-357) over the last N encoder
        states (m1) and the image features (m2 = the same [B, Ti, Di] for every layer)."""
        N = len(states)
        _, Ti, Di = img.shape
        img2 = img.reshape(B * Ti, Di)
        ctx = {"layers": [], "ln1": [], "N": N}
        out = None
        for i in range(N):
            if out is None:
                inp = states[i]
                ctx["ln1"].append(None)
            else:
                s_ = K.add_f16(states[i], out)
                inp, mi, ri = K.layernorm(s_, self.P(EXT + ".layer_norm1.weight"), self.P(EXT + ".layer_norm1.bias"))
                ctx["ln1"].append((s_, mi, ri))
            out, c = self.ext_layer_fwd(i, inp, img2, B, Te, Ti, lens32, img_km)
            ctx["layers"].append(c)
        return out, ctx

    def ext_bwd(self, ctx, dout):
        """-> {i: gradient of the i-th external input state} (i over the N states)."""
        N = ctx["N"]
        d = dout
        out = {}
        # the shared layer_norm1 gradient is summed over the layers above layer 0 (dgb_accumulate;
        # with one layer it is unused and stays 0)
        self.params.span(EXT + ".layer_norm1.weight", EXT + ".layer_norm1.bias", grad=True).zero_()
        for i in reversed(range(N)):
            dinp = self.ext_layer_bwd(i, ctx["layers"][i], d)
            ctx["layers"][i] = None
            if i == 0:
                out[0] = dinp
            else:
                s_, mi, ri = ctx["ln1"][i]
                ds = K.layernorm_bwd(dinp, s_, self.P(EXT + ".layer_norm1.weight"), mi, ri, self._lnspan(EXT + ".layer_norm1"),
                                     dgb_accumulate=True)
                out[i] = ds         # s = m1[i] + out_{i-1}: the same gradient for both
                d = ds
        return out

    # -------------------------------------------------------------- QFormer extractor
    def qformer_fwd(self, enc, img, B, Te, lens32):
        """QFormerModel.forward (fuse.py:829-874, norm None) as mm_s2s_transformer.py:481-486
        calls it: learned queries (query_embedding broadcast over the batch) through the query
        layers (memory = the encoder output enc [B*Te, D], keys masked by the source lengths) and
        the multimodal layers (memory = the image features img [B, Ti, D], unmasked).
        Returns ([B, Q, D], ctx)."""
        D, H, _, Q, nq, nm, saf = qformer_dims(self.cfg)
        pp = self._p("SA_attention_dropout")
        Ti = img.shape[1]
        x = torch.empty(B * Q, D, dtype=F16, device=enc.device)
        K.copy2d(self.P(QF + ".query_embedding").view(1, Q * D).expand(B, Q * D), x.view(B, Q * D), B, Q * D)
        img2 = img.reshape(B * Ti, D)
        ctx = {"q": [], "m": [], "B": B, "Te": Te, "Q": Q}
        for i in range(nq):
            x, c = self.mml_fwd(f"{QF}.query_transformer_layers.{i}", x, enc, B, Q, Te, D, D, H, pp, saf,
                                mem_len=lens32)
            ctx["q"].append(c)
        for i in range(nm):
            x, c = self.mml_fwd(f"{QF}.multimodal_transformer_layers.{i}", x, img2, B, Q, Ti, D, D, H, pp, saf)
            ctx["m"].append(c)
        return x.view(B, Q, D), ctx

    def qformer_bwd(self, ctx, dout, denc):
        """Backward of qformer_fwd: dout [B*Q, D]; the encoder output's gradient is ADDED to denc
        [B*Te, D]; the query embedding's gradient is the batch sum of the first layer's input
        gradient."""
        B, Q = ctx["B"], ctx["Q"]
        d = dout
        for c in reversed(ctx["m"]):
            d = self.mml_bwd(c, d)
        for c in reversed(ctx["q"]):
            d = self.mml_bwd(c, d, dmem=denc, dmem_accumulate=True)
        K.bias_grad(d.view(B, -1), self.G(QF + ".query_embedding").view(-1), side=False)
        return denc

    # -------------------------------------------------------------- decoder layer
    def _sp(self, p):
        return p if self.training else 0.0

    def dec_layer_fwd_ref(self, l, x, kv_all, B, Tt, Te, tgt_mask, enc_len32, tgt_len32=None, spec=None):
        spec = spec or self.dspec
        p = f"{spec.prefix}.layers.{l}"
        d, H = spec.d, spec.H
        hd = d // H
        R = B * Tt
        pd, pa, pact = self._sp(spec.pd), self._sp(spec.pa), self._sp(spec.pact)
        c = {"x": x, "B": B, "Tt": Tt, "Te": Te, "pd": pd, "pa": pa, "pact": pact}
        # self attention (causal + target padding)
        h1, c["m1"], c["r1"] = K.layernorm(x, self.P(p + ".self_attn_layer_norm.weight"), self.P(p + ".self_attn_layer_norm.bias"))
        c["h1"] = h1
        Wqkv = self.params.span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight").view(3 * d, d)
        bqkv = self.params.span(p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias")
        qkv = K.linear(h1, Wqkv, bqkv)
        c["qkv"] = qkv
        O = torch.empty(R, d, dtype=F16, device=x.device)
        c["drop_sa"] = self._drop(pa, B * H * Tt * Tt)
        # right-padded targets: padding == key length (flash path); otherwise the explicit mask
        tgt_len, tmask = (tgt_len32, None) if tgt_len32 is not None else (None, tgt_mask)
        c["sattn"] = attn_forward(qkv, qkv[:, d:], qkv[:, 2 * d:], 3 * d, 3 * d, 3 * d, B, H, Tt, Tt, hd,
                                  hd ** -0.5, O, d, key_len=tgt_len, key_mask=tmask, causal=True, p=pa,
                                  drop=c["drop_sa"])
        c["sO"] = O
        c["drop1"] = self._drop(pd, R * d)
        x2 = K.linear(O, self.P(p + ".self_attn.out_proj.weight"), self.P(p + ".self_attn.out_proj.bias"),
                      epi=K.EPI_DROP_RESID, aux=x, p=pd, drop=c["drop1"])
        c["x2"] = x2
        # encoder attention
        h2, c["m2"], c["r2"] = K.layernorm(x2, self.P(p + ".encoder_attn_layer_norm.weight"), self.P(p + ".encoder_attn_layer_norm.bias"))
        c["h2"] = h2
        q = K.linear(h2, self.P(p + ".encoder_attn.q_proj.weight"), self.P(p + ".encoder_attn.q_proj.bias"))
        ldkv = kv_all.stride(0)
        kv = kv_all[:, 2 * d * l:2 * d * (l + 1)]   # this layer's K | V columns of the batched projection
        c["q"], c["kv"] = q, kv
        O2 = torch.empty(R, d, dtype=F16, device=x.device)
        c["drop_ca"] = self._drop(pa, B * H * Tt * Te)
        c["cattn"] = attn_forward(q, kv, kv[:, d:], d, ldkv, ldkv, B, H, Tt, Te, hd, hd ** -0.5, O2, d,
                                  key_len=enc_len32, p=pa, drop=c["drop_ca"])
        c["cO"] = O2
        c["drop2"] = self._drop(pd, R * d)
        x3 = K.linear(O2, self.P(p + ".encoder_attn.out_proj.weight"), self.P(p + ".encoder_attn.out_proj.bias"),
                      epi=K.EPI_DROP_RESID, aux=x2, p=pd, drop=c["drop2"])
        c["x3"] = x3
        # FFN
        h3, c["m3"], c["r3"] = K.layernorm(x3, self.P(p + ".final_layer_norm.weight"), self.P(p + ".final_layer_norm.bias"))
        c["h3"] = h3
        c["drop_act"] = self._drop(pact, R * spec.F)
        f1 = K.linear(h3, self.P(p + ".fc1.weight"), self.P(p + ".fc1.bias"), epi=K.EPI_RELU_DROP, p=pact,
                      drop=c["drop_act"])
        c["f1"] = f1
        c["drop3"] = self._drop(pd, R * d)
        x4 = K.linear(f1, self.P(p + ".fc2.weight"), self.P(p + ".fc2.bias"), epi=K.EPI_DROP_RESID, aux=x3,
                      p=pd, drop=c["drop3"])
        return x4, c

    def dec_layer_bwd_ref(self, l, c, dx4, dkv_all, dy3=None, emit=None, spec=None):
        """Returns (dx, masked dx for the layer below or None); writes this layer's cross-attention
        K/V gradient into its columns of dkv_all [B*Te, L_d*2d] (the K/V projection's dgrad and
        wgrad run once for all layers, decoder_backward).  dy3/emit as enc_layer_bwd's dy2/emit."""
        spec = spec or self.dspec
        p = f"{spec.prefix}.layers.{l}"
        d, H = spec.d, spec.H
        hd = d // H
        B, Tt, Te = c["B"], c["Tt"], c["Te"]
        pd, pa, pact = c["pd"], c["pa"], c["pact"]
        if dy3 is None:
            dy3 = K.dropout(dx4, pd, c["drop3"], out=torch.empty_like(dx4)) if pd > 0 else dx4
        K.linear_wgrad(dy3, c["f1"], self.G(p + ".fc2.weight"),
                       db=self.G(p + ".fc2.bias"))
        df1 = K.linear_dgrad(dy3, self.P(p + ".fc2.weight"), epi=K.EPI_RELU_DROP_BWD,
                             aux=c["f1"], p=pact)
        K.linear_wgrad(df1, c["h3"], self.G(p + ".fc1.weight"),
                       db=self.G(p + ".fc1.bias"))
        dh3 = K.linear_dgrad(df1, self.P(p + ".fc1.weight"))
        del df1
        dx3, dy2 = K.layernorm_bwd(dh3, c["x3"], self.P(p + ".final_layer_norm.weight"), c["m3"], c["r3"],
                                   self.params.span(p + ".final_layer_norm.weight", p + ".final_layer_norm.bias", grad=True),
                                   dres=dx4, emit=(pd, c["drop2"]))
        # encoder attention
        K.linear_wgrad(dy2, c["cO"], self.G(p + ".encoder_attn.out_proj.weight"),
                       db=self.G(p + ".encoder_attn.out_proj.bias"))
        dO2 = K.linear_dgrad(dy2, self.P(p + ".encoder_attn.out_proj.weight"))
        q, kv = c["q"], c["kv"]
        dq = torch.empty_like(q)
        dkv = dkv_all[:, 2 * d * l:2 * d * (l + 1)]
        ldkv, lddkv = kv.stride(0), dkv.stride(0)
        attn_backward(c["cattn"], dO2, d, c["cO"], q, kv, kv[:, d:], d, ldkv, ldkv, B, H, Tt, Te, hd,
                      hd ** -0.5, dq, dkv, dkv[:, d:], d, lddkv, lddkv, p=pa, drop=c["drop_ca"])
        K.linear_wgrad(dq, c["h2"], self.G(p + ".encoder_attn.q_proj.weight"),
                       db=self.G(p + ".encoder_attn.q_proj.bias"))
        dh2 = K.linear_dgrad(dq, self.P(p + ".encoder_attn.q_proj.weight"))
        dx2, dy1 = K.layernorm_bwd(dh2, c["x2"], self.P(p + ".encoder_attn_layer_norm.weight"), c["m2"], c["r2"],
                                   self.params.span(p + ".encoder_attn_layer_norm.weight", p + ".encoder_attn_layer_norm.bias", grad=True),
                                   dres=dx3, emit=(pd, c["drop1"]))
        # self attention
        K.linear_wgrad(dy1, c["sO"], self.G(p + ".self_attn.out_proj.weight"),
                       db=self.G(p + ".self_attn.out_proj.bias"))
        dO = K.linear_dgrad(dy1, self.P(p + ".self_attn.out_proj.weight"))
        qkv = c["qkv"]
        dqkv = torch.empty_like(qkv)
        attn_backward(c["sattn"], dO, d, c["sO"], qkv, qkv[:, d:], qkv[:, 2 * d:], 3 * d, 3 * d, 3 * d, B, H,
                      Tt, Tt, hd, hd ** -0.5, dqkv, dqkv[:, d:], dqkv[:, 2 * d:], 3 * d, 3 * d, 3 * d, p=pa,
                      drop=c["drop_sa"])
        Wqkv = self.params.span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight").view(3 * d, d)

        def qkv_wgrad():
            K.linear_wgrad(dqkv, c["h1"], self.params.span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight", grad=True).view(3 * d, d),
                           db=self.params.span(p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias", grad=True))
        dh1 = K.linear_dgrad(dqkv, Wqkv)
        qkv_wgrad()
        if emit is None:
            dx = K.layernorm_bwd(dh1, c["x"], self.P(p + ".self_attn_layer_norm.weight"), c["m1"], c["r1"],
                                 self.params.span(p + ".self_attn_layer_norm.weight", p + ".self_attn_layer_norm.bias", grad=True),
                                 dres=dx2)
            return dx, None
        return K.layernorm_bwd(dh1, c["x"], self.P(p + ".self_attn_layer_norm.weight"), c["m1"], c["r1"],
                               self.params.span(p + ".self_attn_layer_norm.weight", p + ".self_attn_layer_norm.bias", grad=True),
                               dres=dx2, emit=emit)

    # -------------------------------------------------------------- full model
    def encoder_forward(self, batch):
        """Returns (enc [B*Te, d], enc_len32, Te, ctx) for a DeviceBatch (runtime.prepare_batch)."""
        cfg = self.cfg
        d = cfg["encoder_embed_dim"]
        src_tokens = batch.src
        imgs, img_mask = batch.imgs, batch.img_keymask
        B = src_tokens.shape[0]
        ctx = {}
        self.params.await_group("sub")
        self.refresh_transposed_weights()
        h, Te, ctx["sub"] = self.subsample_fwd(src_tokens, None)
        assert Te == batch.Te, (Te, batch.Te)
        lens32 = batch.enc_len32
        ctx["lens32"] = lens32
        pos = self._ensure_pos(Te, "enc")
        scale = 1.0 if cfg["no_scale_embedding"] else math.sqrt(d)
        pd = self._p("dropout")
        ctx["drop_emb"] = self._drop(pd, B * Te * d)
        x = K.encoder_embed(h, pos, lens32, B, Te, d, scale, pd, ctx["drop_emb"])
        ctx["emb"] = (scale, pd)
        ctx["layers"] = []
        for l in range(cfg["encoder_layers"]):
            self.params.await_group(f"enc{l}")
            x, c = self.enc_layer_fwd(l, x, B, Te, lens32)
            ctx["layers"].append(c)
        self.params.await_group("enc_tail")
        ctx["lx"] = x
        ctx["fusion"] = None
        ctx["ext"] = None
        if cfg["fusion"] and imgs is not None and cfg["multimodal_attention_type"] == "external_multimodal_transformer":
            # mm_s2s_transformer.py:531-554: the external transformer reads the last N encoder
            # states (the final LayerNorm's output is replaced, so it is not computed) and the raw
            # image features; modality dropout: audio-drop zeroes only the replaced encoder_out
            # (no effect), image-drop zeroes the features (:496-512)
            if self.training:
                mod_p, aud_p = self.np_rng.random(), self.np_rng.random()
                if mod_p < cfg["modality_dropout"] and not aud_p < cfg["audio_dropout"]:
                    imgs = torch.zeros_like(imgs)
            N = cfg["external_multimodal_transformer_layers"]
            states = self.encoder_states(ctx)[-N:]
            out, ctx["ext"] = self.ext_fwd(states, imgs, img_mask, B, Te, lens32)
            ctx["B"], ctx["Te"] = B, Te
            return out, lens32, Te, ctx
        xl, ctx["lm"], ctx["lr"] = K.layernorm(x, self.P("encoder.layer_norm.weight"), self.P("encoder.layer_norm.bias"))
        out = xl
        ctx["qformer"] = None
        if cfg["fusion"] and imgs is not None and cfg["multimodal_extractor_type"] == "q_former":
            # mm_s2s_transformer.py:479-494: the QFormer output replaces the image features before
            # the modality-dropout draws; its Q query tokens are all valid (no image key mask)
            imgs, ctx["qformer"] = self.qformer_fwd(xl, imgs, B, Te, lens32)
            img_mask = None
        if cfg["fusion"] and imgs is not None:
            # modality dropout (mm_s2s_transformer.py:496-512): two host draws every training forward
            if self.training:
                mod_p, aud_p = self.np_rng.random(), self.np_rng.random()
                if mod_p < cfg["modality_dropout"]:
                    if aud_p < cfg["audio_dropout"]:
                        # reference raises UnboundLocalError here; intent: zero audio
                        ctx["audio_dropped"] = True
                        out = torch.zeros_like(xl)
                    else:
                        imgs = torch.zeros_like(imgs)   # LN of zeros -> beta (Q5), as reference
                        ctx["image_dropped"] = True     # (requires_grad=False: no QFormer gradient)
            res, ctx["fusion"] = self.fusion_fwd(out, imgs, img_mask, B, Te)
            out = res
        ctx["B"], ctx["Te"] = B, Te
        return out, lens32, Te, ctx

    def encoder_backward(self, ctx, denc, dstates=None):
        """dstates: {l: gradient of encoder_states[l]} (layer l's output, fairseq's
        ``encoder_states`` with return_all_hiddens) from multitask heads."""
        dstates = dict(dstates or {})
        L = self.cfg["encoder_layers"]
        if ctx.get("ext") is not None:
            N = ctx["ext"]["N"]
            for i, g in self.ext_bwd(ctx["ext"], denc).items():
                l = L - N + i
                dstates[l] = g if l not in dstates else K.add_f16(dstates[l], g)
            self._ready(EXT + ".layer_norm1.bias")
            self._zero_grads(("encoder.layer_norm.",))   # unused by this fusion type: its gradient is 0
            self._ready("encoder.layer_norm.bias")
            return self._encoder_layers_bwd(ctx, dstates.pop(L - 1), None, dstates)
        qf = ctx.get("qformer")
        dimg = None
        if ctx["fusion"] is not None:
            if qf is not None and not ctx.get("image_dropped"):
                denc, dimg = self.fusion_bwd(ctx["fusion"], denc, want_dimg=True)
            else:
                denc = self.fusion_bwd(ctx["fusion"], denc)
                if qf is not None:      # zeroed images (requires_grad=False): no QFormer gradient
                    self._zero_grads((QF + ".",))
            if not self.cfg["use_selective_gate"]:   # built by the reference, unused without the gate
                self._zero_grads(("encoder.gate_denses.",))
        elif self.cfg["fusion"]:        # a batch without image features: the fusion tail did not run
            self._zero_grads(FUSION_PREFIXES)
        if dimg is not None:
            # the QFormer read the (pre-modality-dropout) encoder output as its query layers'
            # memory: that gradient reaches the encoder even when the audio branch was dropped
            if ctx.get("audio_dropped"):
                denc = torch.zeros_like(denc)
            self.qformer_bwd(qf, dimg.view(-1, dimg.shape[-1]), denc)
        last_fusion = [n for n, _ in self.params.specs if n.startswith(FUSION_PREFIXES)]
        if last_fusion:
            self._ready(last_fusion[-1])
        if ctx.get("audio_dropped") and dimg is not None:
            pass    # denc holds the QFormer's memory gradient: the encoder backward runs
        elif ctx.get("audio_dropped") and not dstates:
            # the reference replaces encoder_out by zeros_like(..., requires_grad=False)
            # (mm_s2s_transformer.py:500): no gradient reaches the encoder, whose gradients stay
            # at zero -- skip its whole backward, zero its gradients, flush the reducer
            ctx["layers"] = None
            self._zero_grads(("encoder.layer_norm.", "encoder.transformer_layers.", "encoder.subsample."))
            self._ready(None)
            return
        elif ctx.get("audio_dropped"):
            denc = torch.zeros_like(denc)   # only the multitask heads' state gradients remain
        layers = ctx["layers"]
        emit = lambda l: (layers[l]["pd"], layers[l]["drop2"]) if l >= 0 else None  # noqa: E731
        gln = self.params.span("encoder.layer_norm.weight", "encoder.layer_norm.bias", grad=True)
        if (L - 1) in dstates:     # encoder_states[L-1] = the final LayerNorm's input
            dx = K.layernorm_bwd(denc, ctx["lx"], self.P("encoder.layer_norm.weight"), ctx["lm"], ctx["lr"], gln,
                                 dres=dstates[L - 1])
            dmask = None
        else:
            dx, dmask = K.layernorm_bwd(denc, ctx["lx"], self.P("encoder.layer_norm.weight"), ctx["lm"], ctx["lr"],
                                        gln, emit=emit(L - 1))
        self._ready("encoder.layer_norm.bias")
        return self._encoder_layers_bwd(ctx, dx, dmask, dstates)

    def _encoder_layers_bwd(self, ctx, dx, dmask, dstates):
        """Encoder layers L-1..0, the embedding and the subsampler; dx = gradient of the top
        layer's output, dstates = {l: extra gradient of layer l's output} for l < L-1."""
        layers = ctx["layers"]
        L = self.cfg["encoder_layers"]
        emit = lambda l: (layers[l]["pd"], layers[l]["drop2"]) if l >= 0 else None  # noqa: E731
        for l in reversed(range(L)):
            em = None if (l - 1) in dstates else emit(l - 1)
            dx, dmask = self.enc_layer_bwd(l, layers[l], dx, dy2=dmask, emit=em)
            layers[l] = None
            if (l - 1) in dstates:      # encoder_states[l-1] = this layer's input
                dx = K.add_f16(dx, dstates[l - 1])
                dmask = None
            self._ready(f"encoder.transformer_layers.{l}.self_attn_layer_norm.bias")
        # the last layer's deferred weight-gradient group (layers.hip g_pend) beside the subsampler's
        # backward rather than after it (profiles/round6_wgrad_defer_ab.txt)
        K.wgrad_flush()
        scale, pd = ctx["emb"]
        dh = K.scale_dropout_bwd(dx, scale, pd, ctx["drop_emb"])
        self.subsample_bwd(ctx["sub"], dh)
        self._ready(None)

    def decoder_forward(self, batch, enc, enc_len32, Te, spec=None):
        """fairseq TransformerDecoder (pre-LN, tied output projection) of `spec` (the unit decoder
        by default).  batch: .prev [B, Tt] int64, .tgt_mask, .tgt_len32 (runtime.prepare_batch /
        decoder_batch).  Returns (padded logits [B*Tt, round64(V)], ctx)."""
        spec = spec or self.dspec
        d, V, pad = spec.d, spec.V, spec.pad
        tok = batch.prev
        B, Tt = tok.shape
        ctx = {"B": B, "Tt": Tt, "spec": spec}
        main = spec is self.dspec
        pos = self._ensure_pos(Tt, "dec" if main else d)
        scale = 1.0 if spec.no_scale_embedding else math.sqrt(d)
        pd = self._sp(spec.pd)
        ctx["drop_emb"] = self._drop(pd, B * Tt * d)
        ctx["tok"] = tok
        self.params.await_group("dec_emb" if main else f"aux_{spec.prefix[:-len('_decoder')]}")
        x = K.token_embed(tok, self.P(f"{spec.prefix}.embed_tokens.weight"), pos, B, Tt, d, pad, scale, pd,
                          ctx["drop_emb"])
        ctx["emb"] = (scale, pd)
        tgt_mask = batch.tgt_mask  # uint8 [B, round8(Tt)] or None (no target padding in the batch)
        ctx["layers"] = []
        if main:
            self.params.await_group("cross_kv")
        Wkv, bkv = self.cross_kv(spec=spec)
        kv_all = K.linear(enc, Wkv, bkv)   # [B*Te, L_d*2d]: every layer's cross-attention K | V
        ctx["kv_all"] = kv_all
        for l in range(spec.L):
            if main:
                self.params.await_group(f"dec{l}")
            x, c = self.dec_layer_fwd(l, x, kv_all, B, Tt, Te, tgt_mask, enc_len32, batch.tgt_len32, spec=spec)
            ctx["layers"].append(c)
        if main:
            self.params.await_all()   # "dec_ln" and anything not consumed above
        xl, ctx["lm"], ctx["lr"] = K.layernorm(x, self.P(f"{spec.prefix}.layer_norm.weight"),
                                               self.P(f"{spec.prefix}.layer_norm.bias"))
        ctx["lx"], ctx["xl"] = x, xl
        Vp = round_up(V, 64)  # whole k-tiles for the tied-embedding dgrad (pad columns of dlogits are 0)
        logits = torch.empty(B * Tt, Vp, dtype=F16, device=x.device)
        E = self.P(f"{spec.prefix}.embed_tokens.weight")
        K.gemm(xl, E, logits, B * Tt, V, d, lda=d, ldb=d, ldc=Vp)
        ctx["Vp"] = Vp
        return logits, ctx

    @staticmethod
    def encoder_states(ctx):
        """fairseq ``encoder_states`` (return_all_hiddens) as batch-major [B*Te, d] buffers: every
        encoder layer's output (the last = the final LayerNorm's input)."""
        layers = ctx["layers"]
        return [layers[l + 1]["x"] for l in range(len(layers) - 1)] + ([ctx["lx"]] if layers else [])

    @staticmethod
    def inner_states(ctx):
        """fairseq TransformerDecoder ``inner_states`` as batch-major [B*Tt, d] buffers: the
        embedding output (after dropout), then every layer's output (the last = the final
        LayerNorm's input)."""
        return [c["x"] for c in ctx["layers"]] + [ctx["lx"]]

    def decoder_backward(self, ctx, dlogits, enc, denc, dinner=None, denc_accumulate=False):
        """Hand-written backward of decoder_forward.  denc [B*Te, de] receives the encoder-output
        gradient (added to its contents with denc_accumulate).  dinner: {j: gradient of
        inner_states[j]} from multitask heads reading the decoder's hidden states."""
        spec = ctx["spec"]
        main = spec is self.dspec
        d, V, pad = spec.d, spec.V, spec.pad
        B, Tt = ctx["B"], ctx["Tt"]
        dinner = dinner or {}
        E = self.P(f"{spec.prefix}.embed_tokens.weight")
        dE32 = torch.empty(V, d, dtype=torch.float32, device=E.device)
        # tied output projection: dE = dlogits^T xl ; dxl = dlogits E.  Both halves of the tied
        # embedding gradient (this wgrad and the token scatter below) run on the side stream, in
        # order: the wgrad writes dE32 (no zero fill), the scatter adds to it.
        K.linear_wgrad(dlogits[:, :V], ctx["xl"], None, out_f32=dE32)
        dxl = torch.empty(B * Tt, d, dtype=F16, device=E.device)
        # dxl = dlogits E over K = Vp: E zero-padded to Vp rows (refreshed per step), so the GEMM
        # runs on the LDS-DMA path (K % 64 == 0) instead of the predicated one
        Vp = ctx["Vp"]
        key = ("embed", spec.prefix)
        Ep = self._wpad.get(key)
        if Ep is None or Ep.shape != (Vp, d):
            Ep = torch.zeros(Vp, d, dtype=F16, device=E.device)
            self._wpad[key] = Ep
        K.copy2d(E, Ep, V, d)
        K.gemm(dlogits, Ep, dxl, B * Tt, d, Vp, a_kc=True, b_kc=False, lda=Vp, ldb=d, ldc=d)
        layers = ctx["layers"]
        L = spec.L
        emit = lambda l: (layers[l]["pd"], layers[l]["drop3"]) if l >= 0 else None  # noqa: E731
        gln = self.params.span(f"{spec.prefix}.layer_norm.weight", f"{spec.prefix}.layer_norm.bias", grad=True)
        if L in dinner:      # inner_states[L] = the final LayerNorm's input
            dx = K.layernorm_bwd(dxl, ctx["lx"], self.P(f"{spec.prefix}.layer_norm.weight"), ctx["lm"], ctx["lr"],
                                 gln, dres=dinner[L])
            dmask = None
        else:
            dx, dmask = K.layernorm_bwd(dxl, ctx["lx"], self.P(f"{spec.prefix}.layer_norm.weight"), ctx["lm"],
                                        ctx["lr"], gln, emit=emit(L - 1))
        self._ready(f"{spec.prefix}.layer_norm.bias")
        dkv_all = torch.empty_like(ctx["kv_all"])
        for l in reversed(range(L)):
            em = None if l in dinner else emit(l - 1)     # inner_states[l] = this layer's input
            dx, dmask = self.dec_layer_bwd(l, layers[l], dx, dkv_all, dy3=dmask, emit=em, spec=spec)
            layers[l] = None
            if l in dinner:
                dx = K.add_f16(dx, dinner[l])
                dmask = None      # the layer below recomputes its masked gradient from dx
            self._ready(f"{spec.prefix}.layers.{l}.self_attn_layer_norm.bias")
        K.wgrad_flush()   # the decoder's last deferred group beside the cross-attention K/V products
        # cross-attention K/V projections of all layers: one wgrad (+ bias) and one dgrad (K = L_d*2d)
        Wkv, _ = self.cross_kv(spec=spec)
        gWkv, gbkv = self.cross_kv(grad=True, spec=spec)
        K.linear_wgrad(dkv_all, enc, gWkv, db=gbkv)
        K.linear_dgrad(dkv_all, Wkv, out=denc, accumulate=denc_accumulate)   # the encoder output's gradient
        del dkv_all
        self._ready(f"{spec.prefix}.layers.{L - 1}.encoder_attn.v_proj.bias")
        scale, pd = ctx["emb"]
        gE = self.G(f"{spec.prefix}.embed_tokens.weight")
        with (K.side_begin(dx, ctx["tok"], dE32) or K._NULLCTX):
            K.token_embed_bwd(ctx["tok"], dx, dE32, B, Tt, d, pad, scale, pd, ctx["drop_emb"])
            K.call("mms2ut_splitk_reduce", dE32.data_ptr(), 1, dE32.numel(), V, d, gE.data_ptr(), d, 1, 1.0,
                   K._s())
        self._ready(f"{spec.prefix}.embed_tokens.weight")
