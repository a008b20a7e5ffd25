"""Host runtime: batch preparation (sample dict -> device buffers), the autograd boundary of the
model and of the label-smoothed CE criterion.

The autograd graph has exactly two nodes per step — the whole model and the loss — because the
model's backward is hand-written (model.py); PyTorch only carries the upstream loss-scale
gradient between them.
"""
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import kernels as K
from .kernels import F16, round_up


@dataclass
class DeviceBatch:
    src: torch.Tensor                 # [B, Ts, C] fp16
    src_lengths: torch.Tensor         # [B] int64 (host)
    enc_len32: torch.Tensor           # [B] int32 (device) subsampled lengths
    Te: int
    prev: torch.Tensor                # [B, Tt] int64 (device)
    tgt_mask: Optional[torch.Tensor]  # [B, round8(Tt)] uint8 or None
    tgt_len32: Optional[torch.Tensor]  # [B] int32 non-pad target lengths when right-padded, else None
    target: torch.Tensor              # [B, Tt] int64 (device)
    imgs: Optional[torch.Tensor]      # [B, Ti, Di] fp16 or None
    img_keymask: Optional[torch.Tensor]  # [B, round8(Ti+1)] uint8 or None
    ntokens: int
    nsentences: int
    n_src_frames: int                 # sum of src lengths (the benchmark's unit of work)
    tgt_lengths32: Optional[torch.Tensor] = None   # [B] int32 (device) target lengths (multitask CTC on decoder states)
    mt: Optional[dict] = None         # {task: multitask.MTBatch} (--multitask-config-yaml)


def subsampled_lengths(lengths, n_layers=2):
    """fairseq Conv1dSubsampler.get_out_seq_lens_tensor: floor((L-1)/2)+1 per conv layer."""
    out = np.asarray(lengths, dtype=np.int64).copy()
    for _ in range(n_layers):
        out = (out - 1) // 2 + 1
    return out


def prepare_batch(sample, cfg, device="cuda", src_override=None):
    """fairseq Trainer._prepare_sample (move_to_cuda + apply_half) for the reference's sample
    contract (speech_to_speech_dataset.py:446-468).  Masks/lengths are derived on the host."""
    dev = torch.device(device)
    ni = sample["net_input"]
    lens = ni["src_lengths"].cpu().numpy()
    nl = len(cfg["conv_kernel_sizes"])
    if src_override is None and ni.get("src_tokens") is None and ni.get("src_waves") is not None:
        from .frontend import wave_net_input_src      # waveforms in the sample: GPU fbank front end
        src_override = wave_net_input_src(ni, dev)
    if src_override is not None:
        src = src_override
    else:
        src = ni["src_tokens"].to(dev, non_blocking=True).to(F16)
    Ts = src.shape[1]
    Te = int(subsampled_lengths([Ts], nl)[0])
    enc_len = subsampled_lengths(lens, nl).astype(np.int32)
    prev_cpu = ni["prev_output_tokens"].cpu()
    B, Tt = prev_cpu.shape
    tgt_mask, tgt_len32 = _target_masks(prev_cpu, cfg["padding_idx"], dev)
    imgs = img_keymask = None
    imgs_list = ni.get("imgs_list") or []
    if cfg["fusion"] and len(imgs_list) > 0:
        if len(imgs_list) > 1:
            raise NotImplementedError("one image-feature type (SURVEY Q8)")
        imgs = imgs_list[0].to(dev, non_blocking=True).to(F16)
        masks = ni.get("img_masks_list") or []
        if len(masks) > 0 and masks[0] is not None:
            Ti = imgs.shape[1]
            km = torch.zeros(B, round_up(Ti + 1, 8), dtype=torch.uint8)
            km[:, :Ti] = masks[0].cpu().to(torch.uint8)
            img_keymask = km.to(dev, non_blocking=True)
    tasks = [t for t in (cfg.get("multitask") or []) if t["weight"] != 0]
    mt = None
    if tasks:
        from . import multitask as MT
        if "multitask" not in sample:
            raise ValueError("the model has multitask heads but the sample carries no 'multitask' targets")
        mt = MT.prepare_multitask(sample["multitask"], tasks, dev)
    tl = sample.get("target_lengths")
    if tl is None:
        tl = (~prev_cpu.eq(cfg["padding_idx"])).sum(1)
    return DeviceBatch(
        tgt_lengths32=tl.to(torch.int32).to(dev, non_blocking=True), mt=mt,
        src=src.contiguous(), src_lengths=torch.as_tensor(lens), Te=Te,
        enc_len32=torch.from_numpy(enc_len).to(dev, non_blocking=True),
        prev=prev_cpu.to(dev, non_blocking=True).contiguous(), tgt_mask=tgt_mask, tgt_len32=tgt_len32,
        target=sample["target"].to(dev, non_blocking=True).contiguous(), imgs=imgs,
        img_keymask=img_keymask, ntokens=int(sample["ntokens"]),
        nsentences=int(sample.get("nsentences", B)), n_src_frames=int(lens.sum()))


def _target_masks(prev_cpu, pad, dev):
    """(uint8 [B, round8(Tt)] key mask or None, int32 [B] key lengths when right-padded or None)."""
    B, Tt = prev_cpu.shape
    padm = prev_cpu.eq(pad)
    tgt_mask = None
    if bool(padm.any()):
        tm = torch.zeros(B, round_up(Tt, 8), dtype=torch.uint8)
        tm[:, :Tt] = padm.to(torch.uint8)
        tgt_mask = tm.to(dev, non_blocking=True)
    # fairseq collate_tokens(left_pad=False): padding is a suffix -> it is a key length
    nonpad = (~padm).sum(1)
    right_padded = bool(torch.all(padm == (torch.arange(Tt)[None, :] >= nonpad[:, None])))
    tgt_len32 = nonpad.to(torch.int32).to(dev, non_blocking=True) if right_padded else None
    return tgt_mask, tgt_len32


@dataclass
class DecoderBatch:
    prev: torch.Tensor
    tgt_mask: Optional[torch.Tensor]
    tgt_len32: Optional[torch.Tensor]


def decoder_batch(prev_output_tokens, cfg):
    """The decoder-side fields of a DeviceBatch for a [B, T] prefix already on the device."""
    cpu = prev_output_tokens.cpu()
    dev = prev_output_tokens.device
    tm, tl = _target_masks(cpu, cfg["padding_idx"], dev)
    return DecoderBatch(prev=prev_output_tokens.contiguous(), tgt_mask=tm, tgt_len32=tl)


def _add_state_grads(out, grads):
    """Merge {index: gradient} from the model's exposed hidden-state outputs into ``out``."""
    for j, g in grads.items():
        g = g.to(F16).contiguous()
        out[j] = g if j not in out else K.add_f16(out[j], g)
    return out


class _ModelFn(torch.autograd.Function):
    """Outputs (padded logits, weighted multitask loss fp32 [1]) and, with ``states=True``, the
    hidden states fairseq's ``return_all_hiddens`` exposes as further outputs: the L_e encoder layer
    outputs ([B*Te, d] batch-major; fairseq ``encoder_states``), then the L_d + 1 decoder
    ``inner_states`` ([B*Tt, d]).  Gradients reaching those outputs (e.g. from multitask heads that
    live outside the HIP model, fairseq_adapter.py) enter the hand-written backward where the state
    is produced.  The backward is hand-written: multitask heads on decoder states -> unit decoder ->
    heads on encoder states -> encoder."""

    @staticmethod
    def forward(fctx, anchor, model, batch, states=False):
        from . import multitask as MT
        enc, len32, Te, ectx = model.encoder_forward(batch)
        if getattr(model, "encoder_hook", None) is not None:   # return_all_hiddens (plugins.py)
            model.encoder_hook("enc", enc)
            model.encoder_hook("ctx", ectx)
        logits, dctx = model.decoder_forward(batch, enc, len32, Te)
        aux, actx, alog = MT.aux_forward(model, batch, ectx, dctx, len32, Te)
        model.last_aux_losses = alog
        fctx.model = model
        fctx.saved = (ectx, dctx, enc, batch, actx, Te)
        fctx.bridged = anchor is not model.anchor   # a caller-provided anchor must get a gradient
        if aux is not None:
            aux = aux.reshape(())
        if not states:     # aux: None without multitask heads (no zero tensor per step)
            return logits, aux
        fctx.set_materialize_grads(False)
        es, ins = model.encoder_states(ectx), model.inner_states(dctx)
        fctx.n_enc = len(es)
        return (logits, aux, *es, *ins)

    @staticmethod
    def backward(fctx, dlogits, daux, *dhidden):
        from . import multitask as MT
        model = fctx.model
        ectx, dctx, enc, batch, actx, Te = fctx.saved
        fctx.saved = None
        d = model.cfg["encoder_embed_dim"]
        denc = torch.empty(enc.shape[0], d, dtype=F16, device=enc.device)  # written by decoder_backward
        use_aux = bool(actx) and daux is not None
        if use_aux:
            daux = daux.reshape(1).to(torch.float32).contiguous()
        dinner = MT.aux_backward_decoder_heads(model, actx, daux) if use_aux else {}
        n_enc = getattr(fctx, "n_enc", 0)
        _add_state_grads(dinner, {j: g for j, g in enumerate(dhidden[n_enc:]) if g is not None})
        if dlogits is None:    # only the multitask losses / hidden states were differentiated
            dlogits = torch.zeros(dctx["B"] * dctx["Tt"], dctx["Vp"], dtype=F16, device=enc.device)
        prof = _BWD_PROFILE
        t_cpu = time.thread_time()
        if prof is not None:
            prof.enable()
        model.decoder_backward(dctx, dlogits.contiguous(), enc, denc, dinner=dinner or None)
        del dctx
        dstates = MT.aux_backward_encoder_heads(model, actx, daux, batch.prev.shape[0], Te) if use_aux else {}
        _add_state_grads(dstates, {j: g for j, g in enumerate(dhidden[:n_enc]) if g is not None})
        model.encoder_backward(ectx, denc, dstates or None)
        K.side_join()  # weight gradients (side stream) complete before anyone reads them
        fin = getattr(model, "grad_release_finish", None)
        if fin is not None:     # fairseq_adapter: hand the last parameter groups to autograd
            fin()
        if prof is not None:
            prof.disable()
        BWD_CPU_S[0] += time.thread_time() - t_cpu
        danchor = torch.zeros(1, dtype=torch.float32, device=enc.device) if fctx.bridged else None
        return danchor, None, None, None


# host-side profile of the hand-written backward (it runs on the autograd engine's thread, which a
# profiler enabled on the main thread does not see): bench.py sets a cProfile.Profile here
_BWD_PROFILE = None
# CPU time the backward's issuing thread spent (seconds, summed over calls): bench.py adds it to the
# main thread's CPU time for the host cost per step, which — unlike the wall time to enqueue — does
# not count the host's waits on the runtime
BWD_CPU_S = [0.0]


def model_outputs(model, batch, states=False):
    """(padded logits [B*Tt, round64(V)] fp16, weighted multitask loss fp32 0-dim, or None when the
    model has no multitask heads) — autograd-connected through the hand-written backward.  states=True appends the encoder_states
    and decoder inner_states outputs (see _ModelFn)."""
    return _ModelFn.apply(model.anchor, model, batch, states)


def model_logits(model, batch):
    """Padded logits [B*Tt, round64(V)] fp16 (autograd-connected through the hand-written bwd)."""
    return _ModelFn.apply(model.anchor, model, batch)[0]


class _LSXentFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, logits, target, V, eps, pad, acc):
        rows, ld = logits.shape
        # the kernel writes this call's {loss, nll} (and adds them to acc, the caller's log, if
        # given): no zeroed accumulator, no copies
        out = torch.empty(2, dtype=torch.float32, device=logits.device)
        lse = K.ls_xent_fwd(logits, ld, target, rows, V, eps, pad, acc, call_out=out)
        fctx.saved = (logits, target, lse, V, eps, pad)
        fctx.set_materialize_grads(False)   # no zero-filled gradient for the nll output
        loss, nll = out[0], out[1]
        fctx.mark_non_differentiable(nll)
        return loss, nll

    @staticmethod
    def backward(fctx, gloss, gnll):
        logits, target, lse, V, eps, pad = fctx.saved
        fctx.saved = None
        rows, ld = logits.shape
        g = gloss.reshape(1).to(torch.float32).contiguous()
        # in place: the logits are dead after this point
        K.ls_xent_bwd(logits, ld, target, rows, V, eps, pad, lse, g, logits)
        return logits, None, None, None, None, None


def label_smoothed_ce(logits, target, V, eps, pad, acc=None):
    """fairseq label_smoothed_nll_loss(lprobs=log_softmax(logits.float()), reduce=sum).
    acc: an optional fp32 device [2] (e.g. a trainer's step log) that {loss, nll} are added to."""
    return _LSXentFn.apply(logits, target.reshape(-1), V, eps, pad, acc)
