"""Multitask auxiliary heads (``--multitask-config-yaml``).

The reference trains with ``--multitask-config-yaml config_multitask.yaml``
(mm_s2ut/scripts/textless/1_train.sh:119) and its criterion adds fairseq's multitask losses on
the model's hidden states (mm_s2ut/criterions/speech_to_speech_criterion.py:94-100 ->
fairseq MultitaskCriterion.get_multitask_loss).  Restated here (fairseq un-vendored, unpinned:
parity of these semantics is against this restatement):

* config (fairseq data_cfg MultitaskConfig / SingleTaskConfig): one YAML entry per task with
  ``decoder_type`` (transformer | ctc), ``dict``, ``data``, ``encoder_layer`` or
  ``decoder_layer`` (input_from encoder / decoder, input_layer = that value - 1; encoder default
  -1 = the last layer), ``loss_weight`` (constant), ``decoder_args``, ``label_smoothing`` (0.2)
  and ``zero_infinity`` (True) for the criteria.
* data (fairseq TextTargetMultitaskData): ``{data}/{split}.tsv`` (id, tgt_text), tokens through
  the task dictionary, eos appended except for CTC; collater = right-padded targets, eos-first
  ``prev_output_tokens``, target_lengths, ntokens (speech_to_speech_dataset.py:495-521 reorders
  them with the speech batch).
* heads (fairseq S2STransformerMultitaskModelBase.build_multitask_decoder):
  ``transformer`` -> TransformerDecoder over ``encoder_states[layer]`` with
  base_multitask_text_transformer_decoder_arch defaults (2 layers, d 256, 4 heads, FFN 2048,
  dropout 0.3, attention dropout = dropout, activation dropout 0, tied output projection),
  label-smoothed CE (reduce sum);  ``ctc`` -> CTCDecoder Linear(in_dim, V) on
  ``encoder_states[layer]`` or the unit decoder's ``inner_states[layer]``, fp32 log_softmax,
  F.ctc_loss(reduction sum, blank = <s> = 0).  Total loss = main + sum_t weight_t * loss_t.

On the device every head is HIP: transformer heads reuse the unit decoder's kernels through a
model.DecoderSpec in the same flat parameter buffer (so the optimizer and the bucketed all-reduce
cover them); CTC heads are a GEMM + the csrc/ctc.hip loss kernels.  Their gradients enter the
hand-written backward at the hidden state they read (model.decoder_backward dinner,
model.encoder_backward dstates).
"""
import csv
import os

import numpy as np
import torch

from . import kernels as K
from .kernels import F16, round_up


# ------------------------------------------------------------------------------------ config
def load_multitask_config(path):
    """{task name: raw config dict} in file order (fairseq MultitaskConfig)."""
    import yaml
    with open(path) as f:
        y = yaml.safe_load(f) or {}
    return {k: dict(v or {}) for k, v in y.items()}


def input_spec(raw):
    """(input_from, input_layer) — fairseq SingleTaskConfig.input_from / input_layer."""
    if "decoder_layer" in raw:
        return "decoder", int(raw["decoder_layer"]) - 1
    return "encoder", int(raw.get("encoder_layer", 0)) - 1


def task_model_cfg(name, raw, dictionary, cfg_main):
    """Model-side config of one task (the dict model.param_specs / DecoderSpec.aux read)."""
    dtype = raw.get("decoder_type", "transformer")
    if dtype not in ("transformer", "ctc"):
        raise NotImplementedError(f"multitask decoder_type {dtype!r}")
    for k in ("loss_weight_schedule", "loss_weight_decay_steps", "prepend_bos_and_append_tgt_lang_tag"):
        if raw.get(k):
            raise NotImplementedError(f"multitask option {k}")
    src, layer = input_spec(raw)
    t = {"name": name, "type": dtype, "V": len(dictionary), "pad": dictionary.pad, "eos": dictionary.eos,
         "blank": dictionary.bos, "input_from": src, "layer": layer, "weight": float(raw.get("loss_weight", 0.0)),
         "label_smoothing": float(raw.get("label_smoothing", 0.2)),
         "zero_infinity": bool(raw.get("zero_infinity", True))}
    if dtype == "transformer":
        if src != "encoder":
            raise NotImplementedError("transformer multitask heads read encoder states (fairseq get_multitask_loss)")
        a = dict(raw.get("decoder_args") or {})
        if a.get("share_decoder_input_output_embed", True) is False:
            raise NotImplementedError("untied multitask decoder output projection")
        drop = float(a.get("dropout", 0.3))
        t.update(d=int(a.get("decoder_embed_dim", 256)), H=int(a.get("decoder_attention_heads", 4)),
                 F=int(a.get("decoder_ffn_embed_dim", 2048)), L=int(a.get("decoder_layers", 2)),
                 dropout=drop, attention_dropout=float(a.get("attention_dropout", drop)),
                 activation_dropout=float(a.get("activation_dropout", 0.0)),
                 max_target_positions=int(a.get("max_target_positions", 1024)),
                 no_scale_embedding=bool(a.get("no_scale_embedding", False)))
    L_src = cfg_main["decoder_layers"] + 1 if src == "decoder" else cfg_main["encoder_layers"]
    if not -L_src <= layer < L_src:
        raise ValueError(f"multitask {name}: layer {layer} out of range for {src} ({L_src} states)")
    t["layer"] = layer % L_src
    return t


# ------------------------------------------------------------------------------------ data
class Dictionary:
    """fairseq Dictionary over a dict.txt (``token count`` lines): <s>=0 <pad>=1 </s>=2 <unk>=3."""

    def __init__(self, symbols=()):
        self.symbols = ["<s>", "<pad>", "</s>", "<unk>"]
        self.bos, self.pad, self.eos, self.unk = 0, 1, 2, 3
        self.index = {s: i for i, s in enumerate(self.symbols)}
        for s in symbols:
            self.add(s)

    def add(self, s):
        if s not in self.index:
            self.index[s] = len(self.symbols)
            self.symbols.append(s)
        return self.index[s]

    @classmethod
    def load(cls, path):
        d = cls()
        with open(path, encoding="utf-8") as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                tok = line.rsplit(" ", 1)[0] if " " in line else line
                d.add(tok)
        return d

    def __len__(self):
        return len(self.symbols)

    def encode_line(self, text, append_eos=True):
        """fairseq Dictionary.encode_line(line, add_if_not_exist=False): whitespace tokens."""
        ids = [self.index.get(w, self.unk) for w in text.strip().split()]
        if append_eos:
            ids.append(self.eos)
        return torch.tensor(ids, dtype=torch.long)


class TextTargetMultitaskData:
    """fairseq TextTargetMultitaskData: ``{data}/{split}.tsv`` (columns id, tgt_text)."""

    def __init__(self, data_dir, split, dictionary, decoder_type):
        self.dict = dictionary
        self.append_eos = decoder_type != "ctc"
        self.data = {}
        with open(os.path.join(data_dir, f"{split}.tsv"), encoding="utf-8", newline="") as f:
            for row in csv.DictReader(f, delimiter="\t", quoting=csv.QUOTE_NONE):
                self.data[row["id"]] = row["tgt_text"]

    def get(self, sample_id):
        if sample_id not in self.data:
            return torch.zeros(0, dtype=torch.long)
        return self.dict.encode_line(self.data[sample_id], append_eos=self.append_eos)

    def collater(self, samples):
        return collate_text_targets(samples, self.dict.pad)


def collate_text_targets(samples, pad):
    """TextTargetMultitaskData.collater: collate_tokens(eos_idx=None) for target, and with
    move_eos_to_beginning (the last token rotated to the front) for prev_output_tokens."""
    n = len(samples)
    T = max((int(s.numel()) for s in samples), default=0)
    target = torch.full((n, max(T, 1)), pad, dtype=torch.long)[:, :T]
    prev = target.clone()
    for i, s in enumerate(samples):
        L = int(s.numel())
        target[i, :L] = s
        if L:
            prev[i, 0] = s[-1]
            prev[i, 1:L] = s[:-1]
    return {"target": target, "prev_output_tokens": prev,
            "target_lengths": torch.tensor([int(s.numel()) for s in samples], dtype=torch.long),
            "ntokens": sum(int(s.numel()) for s in samples)}


def sample_multitask(per_task_samples, order):
    """speech_to_speech_dataset.py:495-521: each task's collated targets reordered like the speech
    batch (``order`` = the collater's length sort)."""
    out = {}
    for name, (data, items) in per_task_samples.items():
        tt = data.collater(items)
        out[name] = {"target": tt["target"].index_select(0, order),
                     "target_lengths": tt["target_lengths"].index_select(0, order),
                     "ntokens": tt["ntokens"],
                     "net_input": {"prev_output_tokens": tt["prev_output_tokens"].index_select(0, order)}}
    return out


# ------------------------------------------------------------------------------------ device
class MTBatch:
    """One task's device targets."""
    __slots__ = ("target", "prev", "tgt_mask", "tgt_len32", "ctc_targets", "ctc_len32", "ctc_max", "ntokens")


def prepare_multitask(sample_mt, tasks, device):
    """sample["multitask"] -> {name: MTBatch} on the device (runtime.prepare_batch)."""
    from .runtime import _target_masks
    out = {}
    for t in tasks:
        if t["weight"] == 0:
            continue
        s = sample_mt[t["name"]]
        mb = MTBatch()
        tgt = s["target"]
        mb.ntokens = int(s["ntokens"])
        if t["type"] == "transformer":
            prev = s["net_input"]["prev_output_tokens"]
            mb.prev = prev.to(device).contiguous()
            mb.target = tgt.to(device).contiguous()
            mb.tgt_mask, mb.tgt_len32 = _target_masks(prev.cpu(), t["pad"], device)
        else:
            # CtcCriterion: targets = target[(target != pad) & (target != eos)], lengths = target_lengths
            lens = s["target_lengths"].to(torch.int32)
            keep = (tgt != t["pad"]) & (tgt != t["eos"])
            S = max(int(lens.max()) if lens.numel() else 0, 1)
            ct = torch.zeros(tgt.shape[0], S, dtype=torch.long)
            for i in range(tgt.shape[0]):
                v = tgt[i][keep[i]]
                ct[i, :v.numel()] = v[:S]
            mb.ctc_targets = ct.to(device)
            mb.ctc_len32 = lens.to(device)
            mb.ctc_max = S
        out[t["name"]] = mb
    return out


def aux_forward(model, batch, ectx, dctx, enc_len32, Te):
    """Every active head's forward + loss.  Returns (weighted loss sum fp32 [1] (device) or None,
    per-head contexts, {name: loss tensor [1]})."""
    tasks = [t for t in model.cfg.get("multitask") or [] if t["weight"] != 0]
    if not tasks or batch.mt is None:
        return None, [], {}
    dev = model.device
    total = torch.zeros(1, dtype=torch.float32, device=dev)
    B = batch.prev.shape[0]
    Tt = batch.prev.shape[1]
    enc_states = model.encoder_states(ectx)
    inner = model.inner_states(dctx)
    ctxs, logs = [], {}
    for t in tasks:
        mb = batch.mt[t["name"]]
        lsum = torch.zeros(2, dtype=torch.float32, device=dev)
        c = {"task": t, "mb": mb}
        if t["type"] == "transformer":
            spec = model.aux_specs[t["name"]]
            src = enc_states[t["layer"]]
            logits, c["dctx"] = model.decoder_forward(_DecBatch(mb), src, enc_len32, Te, spec=spec)
            rows, ld = logits.shape
            c["lse"] = K.ls_xent_fwd(logits, ld, mb.target.reshape(-1), rows, spec.V, t["label_smoothing"],
                                     spec.pad, lsum)
            c["logits"], c["src"] = logits, src
        else:
            d = model.cfg["encoder_embed_dim"] if t["input_from"] == "encoder" else model.cfg["decoder_embed_dim"]
            src = enc_states[t["layer"]] if t["input_from"] == "encoder" else inner[t["layer"]]
            T = Te if t["input_from"] == "encoder" else Tt
            in_len = enc_len32 if t["input_from"] == "encoder" else batch.tgt_lengths32
            pre = f"{t['name']}_decoder.proj"
            ld = round_up(t["V"], 8)
            logits = torch.empty(B * T, ld, dtype=F16, device=dev)
            K.linear(src, model.P(pre + ".weight"), model.P(pre + ".bias"), out=logits[:, :t["V"]], ldc=ld)
            c["work"] = K.ctc_loss_fwd(logits, B, T, t["V"], mb.ctc_targets, in_len, mb.ctc_len32, mb.ctc_max,
                                       t["blank"], t["zero_infinity"], lsum[:1])
            c.update(logits=logits, src=src, T=T, in_len=in_len, d=d)
        total += t["weight"] * lsum[:1]
        logs[t["name"]] = lsum[:1]
        ctxs.append(c)
    return total, ctxs, logs


class _DecBatch:
    __slots__ = ("prev", "tgt_mask", "tgt_len32")

    def __init__(self, mb):
        self.prev, self.tgt_mask, self.tgt_len32 = mb.prev, mb.tgt_mask, mb.tgt_len32


def _ctc_backward(model, c, g):
    t = c["task"]
    mb = c["mb"]
    B = c["logits"].shape[0] // c["T"]
    dlog = K.ctc_loss_bwd(c["logits"], B, c["T"], t["V"], mb.ctc_targets, c["in_len"], mb.ctc_len32, mb.ctc_max,
                          t["blank"], c["work"], g)
    pre = f"{t['name']}_decoder.proj"
    V = t["V"]
    K.linear_wgrad(dlog[:, :V], c["src"], model.G(pre + ".weight"))
    if V % 4:
        # the column-sum kernel works on 4-column groups: reduce over the zero-padded width
        db = torch.empty(dlog.shape[1], dtype=F16, device=dlog.device)
        K.bias_grad(dlog, db)
        with (K.side_begin(db) or K._NULLCTX):
            K.copy2d(db.view(1, -1), model.G(pre + ".bias").view(1, V), 1, V)
    else:
        K.bias_grad(dlog[:, :V], model.G(pre + ".bias"))
    model._ready(pre + ".bias")
    return K.linear_dgrad(dlog[:, :V], model.P(pre + ".weight"))


def aux_backward_decoder_heads(model, ctxs, daux):
    """CTC heads on the unit decoder's inner states: {j: d inner_states[j]} (run before the unit
    decoder's backward, which adds them in)."""
    out = {}
    for c in ctxs:
        t = c["task"]
        if t["type"] == "ctc" and t["input_from"] == "decoder":
            g = daux * t["weight"]
            d = _ctc_backward(model, c, g)
            j = t["layer"]
            out[j] = d if j not in out else K.add_f16(out[j], d)
    return out


def aux_backward_encoder_heads(model, ctxs, daux, B, Te):
    """Transformer / CTC heads on encoder states: {l: d encoder_states[l]}."""
    out = {}
    for c in ctxs:
        t = c["task"]
        if t["type"] == "ctc" and t["input_from"] == "decoder":
            continue
        g = daux * t["weight"]
        l = t["layer"]
        if t["type"] == "transformer":
            logits = c["logits"]
            rows, ld = logits.shape
            K.ls_xent_bwd(logits, ld, c["mb"].target.reshape(-1), rows, t["V"], t["label_smoothing"], t["pad"],
                          c["lse"], g, logits)
            acc = l in out
            if not acc:
                out[l] = torch.empty_like(c["src"])
            model.decoder_backward(c["dctx"], logits, c["src"], out[l], denc_accumulate=acc)
        else:
            d = _ctc_backward(model, c, g)
            out[l] = d if l not in out else K.add_f16(out[l], d)
    return out


__all__ = ["load_multitask_config", "task_model_cfg", "Dictionary", "TextTargetMultitaskData",
           "collate_text_targets", "sample_multitask", "prepare_multitask", "aux_forward",
           "aux_backward_decoder_heads", "aux_backward_encoder_heads", "np"]
