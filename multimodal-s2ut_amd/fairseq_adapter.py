"""Registration into fairseq's own registries (``fairseq-train --user-dir multimodal-s2ut_amd``).

fairseq is not importable in this image, so this module is exercised here only against a stub
registry (tests/test_plugins.py); INTEGRATION.md states what a fairseq install must provide.

fairseq's Trainer owns the optimizer: the model exposes ONE ``nn.Parameter`` that aliases the flat
fp16 parameter buffer (model.ParamStore.flat).  Its gradient is the flat gradient buffer, handed to
autograd by the model node's backward, so fairseq's FP16Optimizer/Adam, clip-norm, loss scaler and
DDP all operate on the same bytes the HIP kernels read and write.
"""
import torch

from . import plugins, runtime


class _FlatModelFn(torch.autograd.Function):
    """Model node whose input is the flat parameter: backward returns the flat gradient."""

    @staticmethod
    def forward(fctx, flat, model, batch):
        model.params.grad.zero_()
        enc, len32, Te, ectx = model.encoder_forward(batch)
        logits, dctx = model.decoder_forward(batch, enc, len32, Te)
        fctx.model = model
        fctx.saved = (ectx, dctx, enc, batch)
        return logits

    @staticmethod
    def backward(fctx, dlogits):
        model = fctx.model
        ectx, dctx, enc, batch = fctx.saved
        fctx.saved = None
        denc = torch.zeros(enc.shape[0], model.cfg["encoder_embed_dim"], dtype=enc.dtype, device=enc.device)
        model.decoder_backward(dctx, dlogits.contiguous(), enc, denc)
        del dctx
        model.encoder_backward(ectx, denc)
        from . import kernels as K
        K.side_join()
        return model.params.grad, None, None


def register(fairseq):
    """Register task / model / arch / criterion under the reference's names."""
    from fairseq.criterions import FairseqCriterion, register_criterion
    from fairseq.models import (BaseFairseqModel, register_model, register_model_architecture)
    from fairseq.tasks import FairseqTask, register_task

    @register_task("multimodal_speech_to_speech")
    class FSMultiModalSpeechToSpeechTask(FairseqTask):
        add_args = staticmethod(plugins.MultiModalSpeechToSpeechTask.add_args)

        def __init__(self, args):
            super().__init__(args)
            self.impl = plugins.MultiModalSpeechToSpeechTask(args)

        @classmethod
        def setup_task(cls, args, **kw):
            return cls(args)

        def build_model(self, args, from_checkpoint=False):
            return FSModel(plugins.MM_S2UTTransformerModel.build_model(args, self.impl))

    @register_model("mm_s2ut_transformer")
    class FSModel(BaseFairseqModel):
        def __init__(self, impl):
            super().__init__()
            self.impl = impl
            self.flat = torch.nn.Parameter(impl.net.params.flat, requires_grad=True)

        def forward(self, src_tokens, src_lengths, prev_output_tokens, target=None, **kw):
            sample = {"net_input": {"src_tokens": src_tokens, "src_lengths": src_lengths,
                                    "prev_output_tokens": prev_output_tokens,
                                    "imgs_list": list(kw.get("imgs_list") or []),
                                    "img_masks_list": list(kw.get("img_masks_list") or [])},
                      "target": target if target is not None else prev_output_tokens,
                      "ntokens": int(prev_output_tokens.ne(self.impl.cfg["padding_idx"]).sum())}
            batch = runtime.prepare_batch(sample, self.impl.cfg, self.flat.device)
            logits = _FlatModelFn.apply(self.flat, self.impl.net, batch)
            return logits, {"_batch": batch}

        def train(self, mode=True):
            self.impl.train(mode)
            return super().train(mode)

        # used only when fairseq's own built-in ``speech_to_unit`` criterion wins the name
        def get_normalized_probs(self, net_output, log_probs, sample=None):
            V = self.impl.cfg["vocab_size"]
            B, Tt = net_output[1]["_batch"].prev.shape
            x = net_output[0].view(B, Tt, -1)[:, :, :V].float()
            return torch.log_softmax(x, -1) if log_probs else torch.softmax(x, -1)

        def get_targets(self, sample, net_output):
            return sample["target"]

    register_model_architecture("mm_s2ut_transformer", "mm_s2ut_transformer")(
        plugins.mm_s2ut_architecture_base)

    def _criterion(name):
        @register_criterion(name)
        class FSSpeechToUnit(FairseqCriterion):
            def __init__(self, task, label_smoothing=0.2, sentence_avg=False):
                super().__init__(task)
                self.eps, self.sentence_avg = label_smoothing, sentence_avg

            @staticmethod
            def add_args(parser):
                parser.add_argument("--label-smoothing", type=float, default=0.2)

            def forward(self, model, sample, reduce=True):
                logits, extra = model(**sample["net_input"], target=sample["target"])
                cfg = model.impl.cfg
                loss, nll = runtime.label_smoothed_ce(logits, extra["_batch"].target, cfg["vocab_size"],
                                                      self.eps, cfg["padding_idx"])
                ss = sample["target"].size(0) if self.sentence_avg else sample["ntokens"]
                return loss, ss, {"loss": loss.detach(), "nll_loss": nll.detach(),
                                  "ntokens": sample["ntokens"], "nsentences": sample["target"].size(0),
                                  "sample_size": ss}
        return FSSpeechToUnit

    from fairseq.criterions import CRITERION_REGISTRY
    # fairseq ships its own ``speech_to_unit``; the reference's scripts use that one
    # (1_train.sh:110) and the reference registers only the free names
    crits = {n: _criterion(n) for n in ("speech_to_unit", "speech_to_speech", "speech_to_unit_v2")
             if n not in CRITERION_REGISTRY}
    return FSMultiModalSpeechToSpeechTask, FSModel, crits
