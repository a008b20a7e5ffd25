"""Registration into fairseq's own registries (``fairseq-train --user-dir multimodal-s2ut_amd``).

The reference's calling convention is kept end to end (mm_s2ut/tasks/speech_to_speech.py:45-123,
mm_s2ut/models/mm_s2s_transformer.py:625-700, criterions/speech_to_speech_criterion.py:58-102):

* task ``multimodal_speech_to_speech`` — flags, seeding and the fusion YAML of the reference
  (plugins.MultiModalSpeechToSpeechTask); ``target_dictionary`` = the unit dictionary of
  ``--target-code-size``, ``source_dictionary`` None, ``multitask_tasks`` built the way fairseq's
  SpeechToSpeechTask builds them (MultitaskConfig + DummyMultiTask), ``load_dataset`` -> the
  on-disk manifest as a FairseqDataset (below), ``max_positions``, ``build_generator`` /
  ``inference_step`` -> the HIP beam search.
* model ``mm_s2ut_transformer`` — an nn.Module whose parameters carry the key names of the
  reference's ``MM_S2UTTransformerModel.state_dict()`` (``decoder.output_projection.weight`` tied
  to ``decoder.embed_tokens.weight``, the never-used Q3 projections as persistent buffers).  Every
  parameter is a view into the flat fp16 buffer the HIP kernels read (model.ParamStore.flat), so
  fairseq's FP16Optimizer writing ``p.data`` updates the kernels' weights in place.
  ``forward(src_tokens, src_lengths, prev_output_tokens, ..., return_all_hiddens)`` returns
  ``(logits [B, Tt, V], extra)`` with ``extra["inner_states"]`` and, with return_all_hiddens,
  ``encoder_states`` / ``encoder_padding_mask`` ([T, B, C] views) — autograd-connected: gradients a
  fairseq multitask head puts on them enter the hand-written backward (runtime._ModelFn).
  ``get_normalized_probs([logits], log_probs)`` works on the criterion's one-element list.
  Multitask heads are built by fairseq's own ``build_multitask_decoder`` (as the reference's model
  inherits them) and listed in ``model.multitask_decoders``.
* criteria ``speech_to_speech`` / ``speech_to_unit_v2`` (aliases the reference names) when fairseq
  has not taken the names; fairseq's own ``speech_to_unit`` (the one ``1_train.sh:110`` uses) is
  left in place and drives the model through the convention above.

The dataset hands the waveforms to the model instead of CPU fbank features: ``__getitem__``
reads the WAV (16-bit PCM, ×2^15 as the reference), the collater packs the samples' fp32 bit
patterns as int32 (fairseq's ``apply_half`` converts float32 tensors only) and the model's forward
runs the GPU fbank / CMVN / SpecAugment front end on them (frontend.wave_net_input_src).

fairseq is not importable in this image: tests/fairseq_stub.py restates the fairseq behaviour this
module relies on and tests/test_plugins.py + tests/test_gpu_plugins.py drive the whole path.
"""
import numpy as np
import torch

from . import data as D
from . import manifest as M
from . import plugins, runtime


class _GroupBridge(torch.autograd.Function):
    """The gradient hand-off of one parameter group (a contiguous run of the flat layout, e.g. one
    encoder layer).  Its output is a graph root of its own, not connected to the loss: the
    hand-written backward runs this node's backward re-entrantly (torch.autograd.backward from
    inside runtime._ModelFn.backward) as soon as the group's gradients are final, and the backward
    hands autograd each parameter's view of the flat gradient buffer.  AccumulateGrad adds it into
    ``p.grad`` (fairseq's --update-freq accumulation) and fires torch DDP's per-parameter hook, so
    DDP's bucket all-reduces start while the rest of the backward still runs (fairseq
    distributed_fairseq_model wraps the model in DDP, bucket_cap_mb 25)."""

    @staticmethod
    def forward(fctx, net, names, *params):
        fctx.net, fctx.names = net, names
        return torch.zeros(1, dtype=torch.float32, device=params[0].device)

    @staticmethod
    def backward(fctx, g):
        P = fctx.net.params
        return (None, None, *[P.g[n] for n in fctx.names])


class _LinkedBridge(torch.autograd.Function):
    """The gradient hand-off connected to the loss (``grad_release = "at_end"``): its output is the
    model node's anchor, so the loss graph reaches every parameter through it and the engine runs
    this backward after the model node's backward has filled the flat gradient and joined its side
    stream.  Needed wherever something walks the graph from the loss to the parameters: torch DDP
    with find_unused_parameters (fairseq --find-unused-parameters) or static_graph,
    ``loss.backward(inputs=params)``, ``torch.autograd.grad(loss, params)``."""

    @staticmethod
    def forward(fctx, net, names, *params):
        fctx.net, fctx.names = net, names
        return net.anchor.detach().clone()

    @staticmethod
    def backward(fctx, g):
        P = fctx.net.params
        return (None, None, *[P.g[n] for n in fctx.names])


def _ddp_walks_graph():
    """True inside the forward of a torch DDP wrapper that walks the autograd graph from the outputs
    (find_unused_parameters or static_graph): the per-group bridges' outputs are graph roots of
    their own, so such a DDP would find no parameter behind the loss, mark every one unused and
    then see each marked ready a second time when the groups are released."""
    get = getattr(torch.nn.parallel.DistributedDataParallel, "_get_active_ddp_module", None)
    ddp = get() if get is not None else None
    return ddp is not None and bool(getattr(ddp, "find_unused_parameters", False) or
                                    getattr(ddp, "static_graph", False))


class _GradRelease:
    """Installed as the model's ``grad_ready_hook`` for one forward/backward.  The backward calls
    ``ready(offset)`` each time the flat gradient below ``offset`` is final (after every layer);
    a group is released two ready points later, once the current stream has waited for the
    weight-gradient side stream's work up to that older point (an event recorded then) — so the
    main stream never waits for the layer whose weight gradients are still running beside its
    dgrad chain.  ``finish()`` (after the side stream is joined) releases the rest."""

    LAG = 2

    def __init__(self, net, groups):
        self.net, self.groups = net, list(groups)   # [(end offset, anchor)] in release order
        self.marks = []     # (offset, side-stream event or None) per ready point
        self.next = 0

    def _release(self, upto):
        todo = []
        while self.next < len(self.groups) and self.groups[self.next][0] <= upto:
            todo.append(self.groups[self.next][1])
            self.next += 1
        if todo:
            torch.autograd.backward(todo, [torch.ones_like(a) for a in todo])

    _ring = []   # K.DevEvent, reused round-robin (a wait binds to the record preceding it)

    def ready(self, upto):
        from . import kernels as K
        side = K._Side.stream if K._Side.used else None
        ev = None
        if side is not None:
            ring = _GradRelease._ring
            if len(ring) < self.LAG + 2:
                ring.append(K.DevEvent())
            ev = ring[len(self.marks) % len(ring)].record(side)
        self.marks.append((upto, ev))
        if len(self.marks) > self.LAG:
            off, old = self.marks[-1 - self.LAG]
            if old is not None:
                old.wait(torch.cuda.current_stream())
            self._release(off)

    def finish(self):
        self._release(self.net.params.numel)
        self.net.grad_ready_hook = None
        self.net.grad_release_finish = None


def _module_path(root, dotted):
    """(parent module, leaf name) for a dotted state-dict key, creating empty modules on the way."""
    *path, leaf = dotted.split(".")
    m = root
    for p in path:
        if p not in m._modules:
            m.add_module(p, torch.nn.Module())
        m = m._modules[p]
    return m, leaf


def _fairseq_multitask_tasks(args):
    """fairseq SpeechToSpeechTask.__init__'s multitask set-up (MultitaskConfig + DummyMultiTask)."""
    if not getattr(args, "multitask_config_yaml", None):
        return {}
    from pathlib import Path

    from fairseq.data.audio.data_cfg import MultitaskConfig
    from fairseq.tasks.speech_to_speech import DummyMultiTask
    cfg = MultitaskConfig(Path(args.multitask_config_yaml))
    first = getattr(cfg, "first_pass_decoder_task_index", -1)
    out = {}
    for i, (name, tc) in enumerate(cfg.get_all_tasks().items()):
        out[name] = DummyMultiTask(tc, tc.tgt_dict, first_pass=i == first)
    return out


def register(fairseq):
    """Register task / model / arch / criteria under the reference's names."""
    import fairseq.tasks as fs_tasks
    from fairseq.criterions import CRITERION_REGISTRY, FairseqCriterion, register_criterion
    from fairseq.data import FairseqDataset
    from fairseq.models import BaseFairseqModel, register_model, register_model_architecture
    from fairseq.tasks import register_task
    TaskBase = getattr(fs_tasks, "LegacyFairseqTask", None) or fs_tasks.FairseqTask

    class ManifestDataset(FairseqDataset):
        """One split of the on-disk corpus (manifest.MultiModalS2SManifest) under fairseq's dataset
        contract: items, collater (the reference's sample dict, speech_to_speech_dataset.py:377-471,
        with the waveforms in net_input), sizes / num_tokens / ordered_indices for batch_by_size."""

        def __init__(self, man, seed=1, epoch=1):
            super().__init__()
            self.man, self.seed, self.epoch = man, seed, epoch

        def __len__(self):
            return len(self.man)

        def __getitem__(self, i):
            it = self.man.item(int(i))
            it["wave"] = torch.from_numpy(np.ascontiguousarray(it["wave"], dtype=np.float32).view(np.int32))
            it["id"] = self.man.ids[int(i)]
            return it

        def collater(self, samples):
            if len(samples) == 0:
                return {}
            sample = D.collater(samples)          # no "source": src_tokens None, frames from the WAVs
            by_index = {it["index"]: it for it in samples}
            order = [int(i) for i in sample["id"].tolist()]
            waves = [by_index[i]["wave"] for i in order]
            off = np.concatenate([[0], np.cumsum([w.numel() for w in waves])]).astype(np.int64)
            ni = sample["net_input"]
            ni["src_waves"] = torch.cat(waves)
            ni["src_wave_offsets"] = torch.from_numpy(off)
            ni["src_cmvn"] = bool(self.man.cmvn)
            sa = self.man.specaugment
            if sa is not None and sa.fn + sa.tn > 0:
                rng = np.random.RandomState((self.seed * 1000003 + self.epoch * 7919 + order[0]) % 2 ** 32)
                ni["src_specaugment"] = {"masks": torch.from_numpy(sa.draws(sample["net_input"]["src_lengths"].tolist(),
                                                                           80, rng)),
                                         "n_freq": sa.fn, "n_time": sa.tn, "mask_value": sa.mask_value}
            if self.man.multitask:
                from . import multitask as MT
                pos = {it["index"]: k for k, it in enumerate(samples)}
                perm = torch.tensor([pos[i] for i in order], dtype=torch.long)
                sample["multitask"] = MT.sample_multitask(
                    {n: (d, [d.get(it["id"]) for it in samples]) for n, d in self.man.multitask.items()}, perm)
            return sample

        def num_tokens(self, i):
            return int(self.man.n_frames[i])

        def num_tokens_vec(self, indices):
            return self.man.n_frames[indices]

        def size(self, i):
            return int(self.man.n_frames[i]), int(self.man.tgt_n_frames[i])

        @property
        def sizes(self):
            return self.man.n_frames

        def ordered_indices(self):
            return self.man.ordered_indices(self.seed, self.epoch)

        def set_epoch(self, epoch):
            self.epoch = epoch

        @property
        def supports_prefetch(self):
            return False

        @property
        def can_reuse_epoch_itr_across_epochs(self):
            return False

    @register_task("multimodal_speech_to_speech")
    class FSMultiModalSpeechToSpeechTask(TaskBase):
        add_args = staticmethod(plugins.MultiModalSpeechToSpeechTask.add_args)

        def __init__(self, args):
            super().__init__(args)
            self.impl = plugins.MultiModalSpeechToSpeechTask(args)
            self.tgt_dict = M.UnitDictionary.for_codes(self.impl.vocab_size - 4)
            self.multitask_tasks = _fairseq_multitask_tasks(args)

        @classmethod
        def setup_task(cls, args, **kw):
            return cls(args)

        @property
        def target_dictionary(self):
            return self.tgt_dict

        @property
        def source_dictionary(self):
            return None

        def max_positions(self):
            return (getattr(self.args, "max_source_positions", None) or 6000,
                    getattr(self.args, "max_target_positions", None) or 1024)

        def load_dataset(self, split, epoch=1, combine=False, **kw):
            man = self.impl.load_dataset(split, epoch)
            self.datasets[split] = ManifestDataset(man, seed=getattr(self.args, "seed", 1), epoch=epoch)
            return self.datasets[split]

        def build_model(self, args, from_checkpoint=False):
            return FSModel.build_model(args, self)

        def build_generator(self, models, args, seq_gen_cls=None, extra_gen_cls_kwargs=None, **kw):
            return self.impl.build_generator([m.impl for m in models], args)

        def inference_step(self, generator, models, sample, prefix_tokens=None, constraints=None):
            return self.impl.inference_step(generator, [m.impl for m in models], sample, prefix_tokens, constraints)

    @register_model("mm_s2ut_transformer")
    class FSModel(BaseFairseqModel):
        def __init__(self, impl):
            super().__init__()
            self.impl = impl
            P = impl.net.params
            self._names = list(P.offsets)
            for n in self._names:
                m, leaf = _module_path(self, n)
                m.register_parameter(leaf, torch.nn.Parameter(P.p[n], requires_grad=True))
            for n, t in P.unused.items():          # Q3: in the state dict, never computed
                m, leaf = _module_path(self, n)
                m.register_buffer(leaf, t)
            m, leaf = _module_path(self, "decoder.output_projection.weight")
            m.register_parameter(leaf, self.get_parameter("decoder.embed_tokens.weight"))
            self._params = [self.get_parameter(n) for n in self._names]
            # release groups: the forward-consumption groups of the flat layout, in the order the
            # backward completes them (ascending end offset)
            self._groups = []
            for _, a, b in sorted(P.groups, key=lambda g: g[2]):
                names = [n for n in self._names if a <= P.offsets[n][0] < b]
                if names:   # final once the backward reports its last parameter's end (model._ready)
                    end = max(P.offsets[n][0] + P.offsets[n][2] for n in names)
                    self._groups.append((end, names, [self.get_parameter(n) for n in names]))
            self.encoder_adapter, self.decoder_adapter = impl.encoder, impl.decoder
            self.multitask_decoders = {}
            # "per_group": each parameter group's gradients reach autograd (and torch DDP's bucket
            # hooks) as soon as the hand-written backward has finished them; "at_end": one bridge on
            # the loss path hands every gradient over after the backward (the form for a DDP that
            # walks the graph — chosen automatically for one — and for backward(inputs=...) /
            # autograd.grad over the parameters)
            self.grad_release = "per_group"

        @classmethod
        def build_model(cls, args, task):
            cfg = plugins.cfg_from_args(args, task.impl.multimodal_translation_config, task.impl.vocab_size)
            dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
            model = cls(plugins.MM_S2UTTransformerModel(cfg, device=dev, seed=getattr(args, "seed", 1)))
            if getattr(args, "find_unused_parameters", False):   # fairseq wraps DDP with it
                model.grad_release = "at_end"
            if task.multitask_tasks:
                # fairseq S2STransformerMultitaskModelBase.build_model: one decoder per task on the
                # encoder (or decoder) states, fairseq's own modules
                from fairseq.models import FairseqEncoderModel, FairseqMultiModel
                from fairseq.models.speech_to_speech.s2s_transformer import S2STransformerMultitaskModelBase
                for name, t in task.multitask_tasks.items():
                    in_dim = cfg["encoder_embed_dim"] if t.args.input_from == "encoder" else cfg["decoder_embed_dim"]
                    dec = S2STransformerMultitaskModelBase.build_multitask_decoder(t.args, t.target_dictionary, in_dim)
                    setattr(model, f"{name}_decoder", dec.to(dev))
                    wrap = FairseqEncoderModel if t.args.decoder_type == "ctc" else FairseqMultiModel
                    model.multitask_decoders[name] = wrap(getattr(model, f"{name}_decoder"))
            return model

        def _check_alias(self):
            flat = self.impl.net.params.flat
            lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * flat.element_size()
            for p in (self._params[0], self._params[-1]):
                if not lo <= p.data_ptr() < hi:
                    raise RuntimeError("mm_s2ut_transformer: a parameter no longer aliases the flat HIP buffer "
                                       "(moved to another device or dtype?); build the model on its GPU, in fp16")

        def forward(self, src_tokens, src_lengths, prev_output_tokens, src_audio_path=None, img_path=None,
                    img_tensor=None, imgs_list=(), img_masks_list=(), tgt_speaker=None, return_all_hiddens=False,
                    **kw):
            """mm_s2s_transformer.py:667-700 -> (logits [B, Tt, V], extra)."""
            if tgt_speaker is not None:
                raise NotImplementedError("target speaker embeddings (spk_emb_proj) are out of scope")
            self._check_alias()
            impl, net = self.impl, self.impl.net
            batch = impl._batch(src_tokens, src_lengths, prev_output_tokens, imgs_list, img_masks_list,
                                extra_input=kw)
            anchor = net.anchor
            if torch.is_grad_enabled():
                if self.grad_release not in ("per_group", "at_end"):
                    raise ValueError(f"grad_release must be 'per_group' or 'at_end' (got {self.grad_release!r})")
                if self.grad_release == "per_group" and not _ddp_walks_graph():
                    rel = _GradRelease(net, [(end, _GroupBridge.apply(net, names, *ps))
                                             for end, names, ps in self._groups])
                    net.grad_ready_hook, net.grad_release_finish = rel.ready, rel.finish
                else:
                    anchor = _LinkedBridge.apply(net, self._names, *self._params)
            outs = runtime._ModelFn.apply(anchor, net, batch, True)
            logits = outs[0]
            B, Tt = prev_output_tokens.shape
            cfg = impl.cfg
            V, d, Te, Le = cfg["vocab_size"], cfg["encoder_embed_dim"], batch.Te, cfg["encoder_layers"]
            tm = lambda x, T, c: x.view(B, T, c).transpose(0, 1)  # noqa: E731  batch-major -> [T, B, C]
            extra = {"attn": [None], "_batch": batch, "_logits_padded": logits,
                     "inner_states": [tm(x, Tt, cfg["decoder_embed_dim"]) for x in outs[2 + Le:]]}
            if return_all_hiddens:
                mask = plugins._padding_mask(batch.enc_len32, Te)
                extra["encoder_states"] = [tm(x, Te, d) for x in outs[2:2 + Le]]
                extra["encoder_padding_mask"] = [mask] if bool(mask.any()) else []
            return logits.view(B, Tt, -1)[:, :, :V], extra

        def get_normalized_probs(self, net_output, log_probs, sample=None):
            logits = net_output[0].float()
            return torch.log_softmax(logits, -1) if log_probs else torch.softmax(logits, -1)

        def get_targets(self, sample, net_output):
            return sample["target"]

        def max_positions(self):
            return self.impl.max_positions()

        def max_decoder_positions(self):
            return self.impl.max_decoder_positions()

        def forward_encoder(self, *a, **kw):
            return self.impl.forward_encoder(*a, **kw)

        def reorder_encoder_out(self, encoder_out, new_order):
            return self.impl.reorder_encoder_out(encoder_out, new_order)

        def load_state_dict(self, state_dict, strict=True, model_cfg=None, args=None):
            """fairseq checkpoint_utils.load_checkpoint_to_cpu -> model.load_state_dict: copies into
            the parameter views (i.e. into the flat buffer)."""
            return torch.nn.Module.load_state_dict(self, state_dict, strict=strict)

        def train(self, mode=True):
            self.impl.train(mode)
            return super().train(mode)

    register_model_architecture("mm_s2ut_transformer", "mm_s2ut_transformer")(
        plugins.mm_s2ut_architecture_base)

    def _criterion(name):
        @register_criterion(name)
        class FSSpeechToUnit(FairseqCriterion):
            """speech_to_unit (criterions/speech_to_speech_criterion.py:58-102) with the HIP
            label-smoothed CE (runtime.label_smoothed_ce) on the padded logits; multitask heads
            through the model's multitask_decoders as fairseq's MultitaskCriterion would."""

            def __init__(self, task, label_smoothing=0.2, sentence_avg=False):
                super().__init__(task)
                self.eps, self.sentence_avg = label_smoothing, sentence_avg
                if getattr(task, "multitask_tasks", None):
                    raise NotImplementedError(f"criterion {name}: multitask heads need fairseq's speech_to_unit")

            @staticmethod
            def add_args(parser):
                parser.add_argument("--label-smoothing", type=float, default=0.2)

            def forward(self, model, sample, reduce=True):
                ni = dict(sample["net_input"], return_all_hiddens=True)
                _, extra = model(**ni)
                cfg = model.impl.cfg
                tgt = sample["target"].to(extra["_logits_padded"].device).contiguous()
                loss, nll = runtime.label_smoothed_ce(extra["_logits_padded"], tgt, cfg["vocab_size"], self.eps,
                                                      cfg["padding_idx"])
                ss = sample["target"].size(0) if self.sentence_avg else sample["ntokens"]
                return loss, ss, {"loss": loss.detach(), "nll_loss": nll.detach(),
                                  "ntokens": sample["ntokens"], "nsentences": sample["target"].size(0),
                                  "sample_size": ss}

            @staticmethod
            def logging_outputs_can_be_summed():
                return True
        return FSSpeechToUnit

    # fairseq ships its own ``speech_to_unit``; the reference's scripts use that one
    # (1_train.sh:110), so only the free names are registered here
    crits = {n: _criterion(n) for n in ("speech_to_unit", "speech_to_speech", "speech_to_unit_v2")
             if n not in CRITERION_REGISTRY}
    return FSMultiModalSpeechToSpeechTask, FSModel, crits, ManifestDataset
