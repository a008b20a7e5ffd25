"""fairseq-compatible plugin surface of the reference, backed by the HIP model.

Names, flags and config keys are the reference's:
  task       multimodal_speech_to_speech   mm_s2ut/tasks/speech_to_speech.py:45-123
  model/arch mm_s2ut_transformer           mm_s2ut/models/mm_s2s_transformer.py:625-710
  criterion  speech_to_unit (+ speech_to_speech [README.md:151], speech_to_unit_v2
             [criterions/speech_to_speech_criterion.py:33-35])
  fusion YAML keys                         mm_s2ut/config/multimodal_s2ut_transformer.yaml:1-41

fairseq itself is not importable in this image; the classes register into a local registry with
the same names (``REGISTRY``).  ``fairseq_adapter.py`` re-registers them into fairseq's own
registries when fairseq is importable, so ``fairseq-train --user-dir multimodal-s2ut_amd`` resolves
the same names.
"""
import argparse
import os
import random
from types import SimpleNamespace

import numpy as np
import torch

from . import runtime
from .model import MMS2UTModel, default_cfg

REGISTRY = {"task": {}, "model": {}, "arch": {}, "criterion": {}}


def _register(kind, *names):
    def deco(obj):
        for n in names:
            REGISTRY[kind][n] = obj
        return obj
    return deco


register_task = lambda *n: _register("task", *n)          # noqa: E731
register_model = lambda *n: _register("model", *n)        # noqa: E731
register_criterion = lambda *n: _register("criterion", *n)  # noqa: E731
register_arch = lambda *n: _register("arch", *n)          # noqa: E731


def set_seed(seed=42):
    """tasks/speech_to_speech.py:33-42 (global seeding at task construction)."""
    os.environ["PYTHONHASHSEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


FUSION_KEYS = ("SA_image_dropout", "SA_text_dropout", "SA_attention_dropout", "image_pre_norm",
               "is_fusion_top", "image_feat_path", "image_feat_dim", "flickr30k_root",
               "load_visual_extractor_type", "load_visual_extractor", "modality_dropout",
               "audio_dropout", "multimodal_attention_type", "use_selective_gate", "is_merge_text_img",
               "external_multimodal_transformer_layers")


def load_fusion_yaml(path):
    """The fusion YAML (OmegaConf.load in the reference; yaml.safe_load here — same keys)."""
    import yaml
    with open(path) as f:
        y = yaml.safe_load(f) or {}
    return SimpleNamespace(**{k: y.get(k) for k in set(FUSION_KEYS) | set(y)})

# ------------------------------------------------------------------------------------ arch


def s2ut_architecture_base(args):
    """fairseq s2ut_architecture_base defaults (getattr-with-default; an unset flag is None)."""
    def g(k, v):
        if getattr(args, k, None) is None:
            setattr(args, k, v)
    g("conv_kernel_sizes", "5,5")
    g("conv_channels", 1024)
    g("encoder_embed_dim", 512)
    g("encoder_ffn_embed_dim", 2048)
    g("encoder_layers", 12)
    g("encoder_attention_heads", 8)
    g("encoder_normalize_before", True)
    g("decoder_embed_dim", args.encoder_embed_dim)
    g("decoder_ffn_embed_dim", args.encoder_ffn_embed_dim)
    g("decoder_layers", 6)
    g("decoder_attention_heads", 8)
    g("decoder_normalize_before", True)
    g("decoder_learned_pos", False)
    g("dropout", 0.1)
    g("attention_dropout", args.dropout)
    g("activation_dropout", args.dropout)
    g("activation_fn", "relu")
    g("share_decoder_input_output_embed", False)
    g("no_scale_embedding", False)
    g("decoder_layerdrop", 0.0)
    g("max_source_positions", 6000)
    g("max_target_positions", 1024)
    g("n_frames_per_step", 1)
    g("input_feat_per_channel", 80)
    g("input_channels", 1)


@register_arch("mm_s2ut_transformer")
def mm_s2ut_architecture_base(args):
    """mm_s2s_transformer.py:703-707."""
    s2ut_architecture_base(args)


def cfg_from_args(args, fusion_cfg=None, vocab_size=1004):
    """fairseq args Namespace (+ fusion YAML) -> model config dict."""
    mm_s2ut_architecture_base(args)
    unsupported = []
    if not args.share_decoder_input_output_embed:
        unsupported.append("--share-decoder-input-output-embed is required (tied output projection)")
    if args.activation_fn != "relu":
        unsupported.append("activation_fn must be relu")
    if not (args.encoder_normalize_before and args.decoder_normalize_before):
        unsupported.append("pre-LN (normalize_before) only")
    if args.n_frames_per_step != 1:
        unsupported.append("n_frames_per_step must be 1 (unit targets)")
    if getattr(args, "decoder_learned_pos", False):
        unsupported.append("sinusoidal decoder positions only")
    if unsupported:
        raise NotImplementedError("; ".join(unsupported))
    cfg = default_cfg(
        input_feat_per_channel=args.input_feat_per_channel, input_channels=args.input_channels,
        conv_kernel_sizes=tuple(int(k) for k in str(args.conv_kernel_sizes).split(",")),
        conv_channels=args.conv_channels, encoder_embed_dim=args.encoder_embed_dim,
        encoder_ffn_embed_dim=args.encoder_ffn_embed_dim, encoder_layers=args.encoder_layers,
        encoder_attention_heads=args.encoder_attention_heads, decoder_embed_dim=args.decoder_embed_dim,
        decoder_ffn_embed_dim=args.decoder_ffn_embed_dim, decoder_layers=args.decoder_layers,
        decoder_attention_heads=args.decoder_attention_heads, dropout=args.dropout,
        attention_dropout=args.attention_dropout, activation_dropout=args.activation_dropout,
        vocab_size=vocab_size, max_source_positions=args.max_source_positions,
        max_target_positions=args.max_target_positions, no_scale_embedding=args.no_scale_embedding,
        label_smoothing=getattr(args, "label_smoothing", 0.2), fusion=False)
    if fusion_cfg is not None:
        dims = fusion_cfg.image_feat_dim
        dims = list(dims) if isinstance(dims, (list, tuple)) else [dims]
        if len(dims) != 1:
            raise NotImplementedError("one image-feature type (SURVEY Q8)")
        att = fusion_cfg.multimodal_attention_type
        if att not in ("selective_attention", "multimodal_attention", "external_multimodal_transformer"):
            raise NotImplementedError(f"multimodal_attention_type={att!r} (out of scope: SURVEY §2)")
        extractor = getattr(fusion_cfg, "load_visual_extractor_type", None) or None
        if att == "external_multimodal_transformer" and extractor:
            raise NotImplementedError("on-line visual extractors (ViT / CLIP) are out of scope: pre-extracted features")
        qformer = getattr(fusion_cfg, "multimodal_extractor_type", None) == "q_former"
        if qformer and att == "external_multimodal_transformer":
            raise NotImplementedError("q_former with the external multimodal transformer")
        if getattr(fusion_cfg, "is_merge_text_img", False):
            raise NotImplementedError("is_merge_text_img=True")
        cfg.update(fusion=bool(fusion_cfg.is_fusion_top), multimodal_attention_type=att,
                   use_selective_gate=bool(fusion_cfg.use_selective_gate), image_feat_dim=int(dims[0]),
                   image_pre_norm=bool(fusion_cfg.image_pre_norm),
                   SA_image_dropout=float(fusion_cfg.SA_image_dropout),
                   SA_text_dropout=float(fusion_cfg.SA_text_dropout),
                   SA_attention_dropout=float(fusion_cfg.SA_attention_dropout),
                   modality_dropout=float(fusion_cfg.modality_dropout),
                   audio_dropout=float(fusion_cfg.audio_dropout),
                   external_multimodal_transformer_layers=getattr(fusion_cfg, "external_multimodal_transformer_layers", None))
        if qformer:
            # mm_s2s_transformer.py:194-209 builds the QFormer whenever multimodal_extractor_type is
            # q_former, but calls it (:479-494) only on the on-line visual extractor's output.  With
            # an extractor configured, the image features fed here stand for that (frozen)
            # extractor's last hidden state and run through the QFormer; without one, the QFormer
            # is built and never used (its parameters stay in the state dict, as SURVEY Q3)
            cfg.update(multimodal_extractor_type="q_former" if extractor else None, qformer_unused=not extractor,
                       num_queries=int(getattr(fusion_cfg, "num_queries", 32)),
                       num_query_layers=int(getattr(fusion_cfg, "num_query_layers", 4)),
                       num_multimodal_layers=int(getattr(fusion_cfg, "num_multimodal_layers", 2)),
                       self_attention_first=bool(getattr(fusion_cfg, "self_attention_first", False)))
    return cfg

# ------------------------------------------------------------------------------------ task


@register_task("multimodal_speech_to_speech")
class MultiModalSpeechToSpeechTask:
    """tasks/speech_to_speech.py:45-123 (flags, seeding, fusion/noise YAML loading)."""

    @staticmethod
    def add_args(parser):
        # inherited SpeechToSpeechTask flags used by the canonical command
        parser.add_argument("data", nargs="?", default=None)
        parser.add_argument("--config-yaml", default="config.yaml")
        parser.add_argument("--multitask-config-yaml", default=None)
        parser.add_argument("--target-is-code", action="store_true")
        parser.add_argument("--target-code-size", type=int, default=None)
        parser.add_argument("--n-frames-per-step", type=int, default=1)
        # the reference's own flags (speech_to_speech.py:47-81)
        parser.add_argument("--multimodal-translation-config-yaml", type=str, default=None)
        parser.add_argument("--mhubert-ckpt-path", type=str, default=None)
        parser.add_argument("--wav2vec2-model-dir", type=str, default=None)
        parser.add_argument("--freezing-updates", type=int, default=-1)
        parser.add_argument("--noise-config-yaml", type=str, default=None)

    def __init__(self, args):
        self.args = args
        set_seed(getattr(args, "seed", 1))
        self.multimodal_translation_config = None
        if getattr(args, "multimodal_translation_config_yaml", None):
            self.multimodal_translation_config = load_fusion_yaml(args.multimodal_translation_config_yaml)
        if getattr(args, "mhubert_ckpt_path", None) or getattr(args, "wav2vec2_model_dir", None):
            raise NotImplementedError("pretrained speech encoders are out of scope (SURVEY §2)")
        code_size = getattr(args, "target_code_size", None) or 1000
        self.vocab_size = code_size + 4  # <s> <pad> </s> <unk> + units (fairseq Dictionary)
        self.padding_idx, self.eos = 1, 2
        # fairseq SpeechToSpeechTask: --multitask-config-yaml -> one auxiliary task per entry
        # (dictionary + text targets), SURVEY §8f row 3 (multitask.py)
        self.multitask_tasks = {}
        if getattr(args, "multitask_config_yaml", None):
            from . import multitask as MT
            path = args.multitask_config_yaml
            if not os.path.isabs(path) and getattr(args, "data", None):
                path = os.path.join(args.data, path)
            for name, raw in MT.load_multitask_config(path).items():
                dct = MT.Dictionary.load(raw["dict"])
                self.multitask_tasks[name] = (raw, dct)

    @classmethod
    def setup_task(cls, args, **kw):
        return cls(args)

    def build_model(self, args, device="cuda"):
        return MM_S2UTTransformerModel.build_model(args, self, device=device)

    def multitask_model_cfg(self, cfg):
        """Model-side configs of the tasks with a non-zero loss weight (fairseq skips the others)."""
        from . import multitask as MT
        out = []
        for name, (raw, dct) in self.multitask_tasks.items():
            t = MT.task_model_cfg(name, raw, dct, cfg)
            if t["weight"] != 0:
                out.append(t)
        return out

    def build_criterion(self, args):
        return SpeechToUnitCriterion(self, getattr(args, "label_smoothing", 0.2))

    def load_dataset(self, split, epoch=1, **kw):
        """speech_to_speech.py:100-123 -> the on-disk manifest (manifest.MultiModalS2SManifest)."""
        import os

        from . import manifest as M
        a = self.args
        fus = self.multimodal_translation_config
        data_cfg = M.load_data_config(os.path.join(a.data, getattr(a, "config_yaml", "config.yaml")))
        feat = getattr(fus, "image_feat_path", None) if fus is not None else None
        if not hasattr(self, "datasets"):
            self.datasets = {}
        self.datasets[split] = M.MultiModalS2SManifest(
            a.data, split, M.UnitDictionary.for_codes(self.vocab_size - 4), data_cfg=data_cfg,
            image_feat_path=feat, is_train=split.startswith("train"),
            max_source_positions=getattr(a, "max_source_positions", None) or 6000,
            max_target_positions=getattr(a, "max_target_positions", None) or 1024,
            multitask=self.multitask_tasks or None)
        return self.datasets[split]

    def build_generator(self, models, args, **kw):
        """fairseq SpeechToSpeechTask.build_generator for unit targets: beam search
        (--beam, --max-len-a, --max-len-b, --lenpen, --min-len; 2_inference.sh:34-44)."""
        return UnitSequenceGenerator(models, beam_size=getattr(args, "beam", 5),
                                     max_len_a=getattr(args, "max_len_a", 0.0),
                                     max_len_b=getattr(args, "max_len_b", 200),
                                     len_penalty=getattr(args, "lenpen", 1.0),
                                     min_len=getattr(args, "min_len", 1))

    def inference_step(self, generator, models, sample, prefix_tokens=None, constraints=None):
        if prefix_tokens is not None or constraints is not None:
            raise NotImplementedError("prefix tokens / constraints in beam search")
        return generator.generate(models, sample)


class UnitSequenceGenerator:
    """fairseq SequenceGenerator surface (``generate(models, sample)`` -> per sentence, hypotheses
    sorted by score: {"tokens", "score", "attention", "alignment", "positional_scores"}) over
    generate.IncrementalDecoder (HIP) + generate.SequenceGenerator."""

    def __init__(self, models, beam_size=5, max_len_a=0.0, max_len_b=200, len_penalty=1.0, min_len=1):
        if len(models) != 1:
            raise NotImplementedError("ensembles in beam search")
        self.model = models[0]
        self.beam_size, self.max_len_a, self.max_len_b = beam_size, max_len_a, max_len_b
        self.len_penalty, self.min_len = len_penalty, min_len

    def generate(self, models, sample, **kw):
        from . import generate as G
        net = (models[0] if models else self.model).net
        batch = runtime.prepare_batch(sample, net.cfg, net.device)
        hyps = G.generate(net, batch, self.beam_size, self.max_len_a, self.max_len_b,
                          len_penalty=self.len_penalty, min_len=self.min_len)
        for hs in hyps:
            for h in hs:
                h["attention"], h["alignment"] = None, None
        return hyps

# ------------------------------------------------------------------------------------ model


def _padding_mask(len32, Te):
    """bool [B, Te] (True = pad) from subsampled lengths (fairseq lengths_to_padding_mask)."""
    return torch.arange(Te, device=len32.device)[None, :] >= len32.long()[:, None]


def encoder_out_dict(net, enc, len32, Te, ctx=None, return_all_hiddens=False):
    """fairseq S2TTransformerEncoder's output contract over the HIP encoder's
    batch-major buffers, as zero-copy time-major views: encoder_out [Te, B, C]; encoder_padding_mask
    [B, Te] or [] when nothing is padded (fairseq's idiom); encoder_states: the L_e
    layer outputs before the final LayerNorm when return_all_hiddens (else [])."""
    d = net.cfg["encoder_embed_dim"]
    B = len32.shape[0]
    tm = lambda x: x.view(B, Te, d).transpose(0, 1)  # noqa: E731
    mask = _padding_mask(len32, Te)
    states = []
    if return_all_hiddens and ctx is not None:
        layers = ctx["layers"]
        states = [tm(layers[l + 1]["x"]) for l in range(len(layers) - 1)] + ([tm(ctx["lx"])] if layers else [])
    return {"encoder_out": [tm(enc)], "encoder_padding_mask": [mask] if bool(mask.any()) else [],
            "encoder_embedding": [], "encoder_states": states, "src_tokens": [], "src_lengths": []}


def reorder_encoder_out(encoder_out, new_order):
    """fairseq S2TTransformerEncoder.reorder_encoder_out: select batch entries (beam expansion /
    finished sentences leaving the batch) in every field of the encoder-out dict."""
    sel = lambda xs, dim: [x.index_select(dim, new_order) for x in xs]  # noqa: E731
    return {"encoder_out": sel(encoder_out["encoder_out"], 1),
            "encoder_padding_mask": sel(encoder_out["encoder_padding_mask"], 0),
            "encoder_embedding": sel(encoder_out.get("encoder_embedding", []), 0),
            "encoder_states": sel(encoder_out.get("encoder_states", []), 1),
            "src_tokens": [], "src_lengths": []}


def _enc_from_dict(net, encoder_out):
    """encoder-out dict -> (batch-major fp16 [B*Te, d], subsampled lengths int32 [B], Te)."""
    x = encoder_out["encoder_out"][0]
    Te, B, d = x.shape
    enc = x.transpose(0, 1).to(torch.float16).contiguous().view(B * Te, d)
    pm = encoder_out.get("encoder_padding_mask") or []
    if len(pm) > 0:
        len32 = (~pm[0]).sum(1).to(torch.int32)
    else:
        len32 = torch.full((B,), Te, dtype=torch.int32, device=x.device)
    return enc, len32.contiguous(), Te


class EncoderAdapter:
    """``model.encoder`` as fairseq's generator drives it: forward / forward_torchscript /
    reorder_encoder_out / max_positions (MM_S2STransformerEncoder, mm_s2s_transformer.py:378-562)."""

    def __init__(self, owner):
        self.owner = owner

    def forward(self, src_tokens, src_lengths, src_audio_path=None, img_path=None, img_tensor=None,
                imgs_list=(), img_masks_list=(), tgt_speaker=None, return_all_hiddens=False, **kw):
        return self.owner.forward_encoder(src_tokens, src_lengths, src_audio_path, img_path, img_tensor,
                                          imgs_list, img_masks_list, tgt_speaker, return_all_hiddens)

    __call__ = forward

    def forward_torchscript(self, net_input):
        return self.forward(**{k: v for k, v in net_input.items() if k != "prev_output_tokens"})

    def reorder_encoder_out(self, encoder_out, new_order):
        return reorder_encoder_out(encoder_out, new_order)

    def max_positions(self):
        return self.owner.cfg["max_source_positions"]


class DecoderAdapter:
    """``model.decoder`` with fairseq's incremental-decoder interface (TransformerUnitDecoder):
    forward(prev_output_tokens, encoder_out, incremental_state) -> (logits [B, T, V], extra),
    reorder_incremental_state(_scripting), get_normalized_probs, max_positions.  Without an
    incremental_state the whole prefix is decoded (teacher forcing); with one, the HIP incremental
    decoder (generate.IncrementalDecoder: KV cache + slot table) decodes the last position."""

    KEY = "_mms2ut_incremental_decoder"

    def __init__(self, owner):
        self.owner = owner

    def forward(self, prev_output_tokens, encoder_out=None, incremental_state=None, features_only=False, **kw):
        net = self.owner.net
        if features_only:
            raise NotImplementedError("features_only decoder outputs")
        if torch.is_grad_enabled() and net.training:
            raise NotImplementedError("decoder adapter is inference-only: training runs the fused model "
                                      "forward (its backward is hand-written end to end)")
        V = self.owner.cfg["vocab_size"]
        enc, len32, Te = _enc_from_dict(net, encoder_out)
        tok = prev_output_tokens.to(enc.device)
        B, T = tok.shape
        if incremental_state is None:
            batch = runtime.decoder_batch(tok, self.owner.cfg)
            with torch.no_grad():
                logits, _ = net.decoder_forward(batch, enc, len32, Te)
            return logits.view(B, T, -1)[:, :, :V].float(), {"attn": [None], "inner_states": None}
        from . import generate as G
        inc = incremental_state.get(self.KEY)
        if inc is None:
            if T != 1:
                raise NotImplementedError("incremental decoding must start from the first position")
            maxlen = int(os.environ.get("MMS2UT_INC_MAXLEN", min(1024, self.owner.cfg["max_target_positions"])))
            inc = G.IncrementalDecoder(net, enc, len32, Te, B, 1, maxlen)
            incremental_state[self.KEY] = inc
        with torch.no_grad():
            inc.step(tok[:, -1].contiguous(), T - 1)
        return inc.logits[:, :V].float().view(B, 1, V), {"attn": [None], "inner_states": None}

    __call__ = forward

    def reorder_incremental_state(self, incremental_state, new_order):
        inc = incremental_state.get(self.KEY) if incremental_state is not None else None
        if inc is not None:
            # beam = 1 inside: every hypothesis owns its encoder rows, gathered with it
            inc.reorder(new_order.to(inc.dev), batch_idxs=new_order.to(inc.dev))

    reorder_incremental_state_scripting = reorder_incremental_state

    def get_normalized_probs(self, net_output, log_probs, sample=None):
        logits = net_output[0].float()
        return torch.log_softmax(logits, -1) if log_probs else torch.softmax(logits, -1)

    def max_positions(self):
        return self.owner.cfg["max_target_positions"]


@register_model("mm_s2ut_transformer")
class MM_S2UTTransformerModel:
    """mm_s2s_transformer.py:625-700 over the HIP model (module tree / state-dict keys kept)."""

    def __init__(self, cfg, device="cuda", seed=1):
        self.net = MMS2UTModel(cfg, device=device, seed=seed).init_params(seed)
        self.cfg = self.net.cfg
        self.encoder = EncoderAdapter(self)
        self.decoder = DecoderAdapter(self)

    @classmethod
    def build_model(cls, args, task, device="cuda"):
        cfg = cfg_from_args(args, task.multimodal_translation_config, task.vocab_size)
        if getattr(task, "multitask_tasks", None):
            cfg["multitask"] = task.multitask_model_cfg(cfg)
        return cls(cfg, device=device, seed=getattr(args, "seed", 1))

    def train(self, mode=True):
        self.net.train(mode)
        return self

    def eval(self):
        return self.train(False)

    def state_dict(self):
        return self.net.params.state_dict()

    def load_state_dict(self, sd, strict=True):
        sd = {k: v for k, v in sd.items() if k != "decoder.output_projection.weight"}
        return self.net.params.load_state_dict(sd, strict=strict)

    def max_positions(self):
        return (self.cfg["max_source_positions"], self.cfg["max_target_positions"])

    def max_decoder_positions(self):
        return self.cfg["max_target_positions"]

    def _batch(self, src_tokens, src_lengths, prev_output_tokens, imgs_list, img_masks_list, target=None,
               multitask=None, extra_input=None):
        """extra_input: further net_input keys (the waveform front-end fields, frontend.wave_net_input_src)."""
        ni = {k: v for k, v in (extra_input or {}).items() if k.startswith("src_")}
        sample = {"net_input": {**ni, "src_tokens": src_tokens, "src_lengths": src_lengths,
                                "prev_output_tokens": prev_output_tokens, "imgs_list": list(imgs_list or []),
                                "img_masks_list": list(img_masks_list or [])},
                  "target": target if target is not None else prev_output_tokens,
                  "ntokens": int(prev_output_tokens.ne(self.cfg["padding_idx"]).sum())}
        cfg = self.cfg
        if multitask is not None:
            sample["multitask"] = multitask
        elif cfg.get("multitask"):
            cfg = dict(cfg, multitask=None)    # inference / no multitask targets: heads unused
        return runtime.prepare_batch(sample, cfg, self.net.device)

    def forward_encoder(self, src_tokens, src_lengths, src_audio_path=None, img_path=None, img_tensor=None,
                        imgs_list=(), img_masks_list=(), tgt_speaker=None, return_all_hiddens=False, **kw):
        """mm_s2s_transformer.py:643-665 -> fairseq's encoder-out dict (encoder_out_dict).  The
        encoder runs without a tape (inference / generation); training gradients flow through
        ``forward``, whose backward is hand-written across the whole model."""
        if tgt_speaker is not None:
            raise NotImplementedError("target speaker embeddings (spk_emb_proj) are out of scope")
        B = src_tokens.shape[0]
        prev = torch.full((B, 1), 2, dtype=torch.long)
        batch = self._batch(src_tokens, src_lengths, prev, imgs_list, img_masks_list)
        with torch.no_grad():
            enc, len32, Te, ctx = self.net.encoder_forward(batch)
        return encoder_out_dict(self.net, enc, len32, Te, ctx, return_all_hiddens)

    def reorder_encoder_out(self, encoder_out, new_order):
        return reorder_encoder_out(encoder_out, new_order)

    def reorder_incremental_state(self, incremental_state, new_order):
        self.decoder.reorder_incremental_state(incremental_state, new_order)

    def get_normalized_probs(self, net_output, log_probs, sample=None):
        return self.decoder.get_normalized_probs(net_output, log_probs, sample)

    def forward(self, src_tokens, src_lengths, prev_output_tokens, src_audio_path=None, img_path=None,
                img_tensor=None, imgs_list=(), img_masks_list=(), tgt_speaker=None,
                return_all_hiddens=False, target=None, multitask=None, **kwargs):
        """Reference signature (mm_s2s_transformer.py:667-680) -> (logits [B, Tt, V], extra).
        The logits are autograd-connected to the hand-written backward.  return_all_hiddens adds
        ``encoder_states`` (L_e layer outputs, [Te, B, C]) and ``encoder_padding_mask`` to extra
        as the reference does (:697-699)."""
        if tgt_speaker is not None:
            raise NotImplementedError("target speaker embeddings (spk_emb_proj) are out of scope")
        batch = self._batch(src_tokens, src_lengths, prev_output_tokens, imgs_list, img_masks_list, target,
                            multitask, extra_input=kwargs)
        stash = {}
        if return_all_hiddens:
            self.net.encoder_hook = stash.__setitem__
        try:
            logits, aux = runtime.model_outputs(self.net, batch)
        finally:
            self.net.encoder_hook = None
        B, Tt = prev_output_tokens.shape
        V = self.cfg["vocab_size"]
        out = logits.view(B, Tt, -1)[:, :, :V]
        extra = {"attn": [None], "inner_states": None, "_batch": batch, "_logits_padded": logits, "_aux_loss": aux}
        if return_all_hiddens:
            eo = encoder_out_dict(self.net, stash["enc"], batch.enc_len32, batch.Te, stash["ctx"], True)
            extra["encoder_states"] = eo["encoder_states"]
            extra["encoder_padding_mask"] = eo["encoder_padding_mask"]
        return out, extra

    __call__ = forward

# ------------------------------------------------------------------------------------ criterion


@register_criterion("speech_to_unit", "speech_to_speech", "speech_to_unit_v2")
class SpeechToUnitCriterion:
    """fairseq speech_to_unit (ref copy criterions/speech_to_speech_criterion.py:58-102):
    label-smoothed NLL (eps), reduce=sum, sample_size = ntokens (sentence_avg False)."""

    def __init__(self, task, label_smoothing=0.2, sentence_avg=False):
        self.eps = label_smoothing
        self.sentence_avg = sentence_avg
        self.padding_idx = getattr(task, "padding_idx", 1)

    def __call__(self, model, sample, reduce=True):
        return self.forward(model, sample, reduce)

    def forward(self, model, sample, reduce=True):
        ni = dict(sample["net_input"])
        _, extra = model(**ni, target=sample["target"], multitask=sample.get("multitask"))
        batch, logits = extra["_batch"], extra["_logits_padded"]
        loss, nll = runtime.label_smoothed_ce(logits, batch.target, model.cfg["vocab_size"], self.eps,
                                              self.padding_idx)
        sample_size = sample["target"].size(0) if self.sentence_avg else sample["ntokens"]
        logging_output = {"loss": loss.detach(), "nll_loss": nll.detach(), "ntokens": sample["ntokens"],
                          "nsentences": sample["target"].size(0), "sample_size": sample_size}
        if model.cfg.get("multitask"):
            # fairseq SpeechToUnitMultitaskTaskCriterion: loss += sum_t weight_t * loss_t; the logged
            # "loss" is the main one, the heads are logged under "multitask"
            loss = loss + extra["_aux_loss"]
            logging_output["multitask"] = {k: {"loss": v.detach(), "loss_weight": w}
                                           for (k, v), w in zip(model.net.last_aux_losses.items(),
                                                                [t["weight"] for t in model.cfg["multitask"]])}
        return loss, sample_size, logging_output

    @staticmethod
    def logging_outputs_can_be_summed():
        # fixed scalars: summed with one all-reduce (parallel.all_reduce_scalars), unlike the
        # reference's all_gather_list
        return True


def build_parser():
    """Flag subset of the canonical command (scripts/textless/1_train.sh:105-125)."""
    p = argparse.ArgumentParser("mms2ut-train")
    MultiModalSpeechToSpeechTask.add_args(p)
    p.add_argument("--task", default="multimodal_speech_to_speech")
    p.add_argument("--arch", default="mm_s2ut_transformer")
    p.add_argument("--criterion", default="speech_to_unit")
    p.add_argument("--label-smoothing", type=float, default=0.2)
    p.add_argument("--share-decoder-input-output-embed", action="store_true")
    p.add_argument("--dropout", type=float, default=0.1)
    p.add_argument("--attention-dropout", type=float, default=0.1)
    p.add_argument("--relu-dropout", dest="activation_dropout", type=float, default=0.1)
    p.add_argument("--activation-dropout", dest="activation_dropout", type=float)
    # architecture flags: None = the arch default (s2ut_architecture_base)
    for f, t in (("--conv-kernel-sizes", str), ("--conv-channels", int), ("--encoder-embed-dim", int),
                 ("--encoder-ffn-embed-dim", int), ("--encoder-layers", int),
                 ("--encoder-attention-heads", int), ("--decoder-embed-dim", int),
                 ("--decoder-ffn-embed-dim", int), ("--decoder-layers", int),
                 ("--decoder-attention-heads", int)):
        p.add_argument(f, type=t, default=None)
    p.add_argument("--lr", type=float, default=5e-4)
    p.add_argument("--lr-scheduler", default="inverse_sqrt")
    p.add_argument("--warmup-init-lr", type=float, default=1e-7)
    p.add_argument("--warmup-updates", type=int, default=10000)
    p.add_argument("--optimizer", default="adam")
    p.add_argument("--adam-betas", default="(0.9,0.98)")
    p.add_argument("--clip-norm", type=float, default=10.0)
    p.add_argument("--max-update", type=int, default=100)
    p.add_argument("--max-tokens", type=int, default=40000)
    p.add_argument("--update-freq", type=int, default=1)
    p.add_argument("--max-target-positions", type=int, default=None)
    p.add_argument("--max-source-positions", type=int, default=None)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--fp16", action="store_true")
    p.add_argument("--fp16-init-scale", type=int, default=128)
    p.add_argument("--num-workers", type=int, default=0)
    p.add_argument("--user-dir", default=None)
    p.add_argument("--save-dir", default=None)
    p.add_argument("--restore-file", default="checkpoint_last.pt")
    p.add_argument("--save-interval-updates", type=int, default=0)
    p.add_argument("--log-interval", type=int, default=10)
    # accepted for command-line compatibility with 1_train.sh (no effect on the training step)
    p.add_argument("--distributed-world-size", type=int, default=None)
    p.add_argument("--tensorboard-logdir", default=None)
    p.add_argument("--vocoder", default=None)
    p.add_argument("--train-subset", default="train")
    p.add_argument("--valid-subset", default="valid")
    p.add_argument("--gen-subset", default="test")
    p.add_argument("--required-batch-size-multiple", type=int, default=1)
    p.add_argument("--synthetic", action="store_true", help="synthetic Speech-Multi30K-shaped data")
    p.add_argument("--no-balanced-sharding", dest="balanced_sharding", action="store_false",
                   help="deal batches to DP ranks round-robin (fairseq ShardedIterator) instead of in "
                        "groups of equal padded cost (SURVEY 8e token-balanced sharding)")
    # fairseq-generate (scripts/textless/2_inference.sh:34-44)
    p.add_argument("--beam", type=int, default=5)
    p.add_argument("--max-len-a", type=float, default=0.0)
    p.add_argument("--max-len-b", type=int, default=200)
    p.add_argument("--lenpen", type=float, default=1.0)
    p.add_argument("--min-len", type=int, default=1)
    return p
