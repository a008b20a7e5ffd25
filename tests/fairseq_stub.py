"""A stand-in for the parts of fairseq that ``fairseq_adapter.py`` is driven by (test
infrastructure; fairseq is un-vendored and absent here).  Each piece restates the
behaviour of the fairseq API it replaces, so a test can run the fairseq-train call sequence
setup_task -> load_dataset -> build_model -> build_criterion -> batches -> criterion -> backward
against the adapter:

* ``fairseq.tasks`` — LegacyFairseqTask: abstract ``load_dataset`` / dictionaries raise,
  ``build_model`` through the arch registry, ``build_criterion`` with FairseqCriterion's
  argument inference, ``get_batch_iterator`` = set_epoch -> ordered_indices ->
  filter_indices_by_size -> batch_by_size -> collater (no worker processes).
* ``fairseq.data`` — FairseqDataset's ``batch_by_size`` (data_utils.batch_by_size, num_tokens
  = the dataset's) and ``filter_indices_by_size``.
* ``fairseq.models`` — BaseFairseqModel, the model / arch registries, FairseqEncoderModel
  (multitask CTC wrapper), ``speech_to_speech.s2s_transformer.S2STransformerMultitaskModelBase.
  build_multitask_decoder`` (ctc: CTCDecoder = Linear(in_dim, |dict|)).
* ``fairseq.criterions`` — FairseqCriterion, the registry and the built-in ``speech_to_unit``
  criterion: the reference's forward (mm_s2ut/criterions/speech_to_speech_criterion.py:58-102,
  rdrop 0) + LabelSmoothedCrossEntropyCriterion.compute_loss (get_normalized_probs on
  ``[net_output]``, label_smoothed_nll_loss, reduce sum) + MultitaskCriterion.get_multitask_loss
  for CTC heads on encoder states + CtcCriterion (fp32 log-softmax, F.ctc_loss sum).
* ``fairseq.data.audio.data_cfg.MultitaskConfig`` / ``fairseq.tasks.speech_to_speech.DummyMultiTask``.
* ``fairseq.utils`` — move_to_cuda / apply_half (Trainer._prepare_sample).
"""
import inspect
import sys
import types
from argparse import Namespace

import numpy as np
import torch
import torch.nn.functional as F


def _label_smoothed_nll_loss(lprobs, target, epsilon, ignore_index=None, reduce=True):
    """fairseq.criterions.label_smoothed_cross_entropy.label_smoothed_nll_loss."""
    if target.dim() == lprobs.dim() - 1:
        target = target.unsqueeze(-1)
    nll_loss = -lprobs.gather(dim=-1, index=target)
    smooth_loss = -lprobs.sum(dim=-1, keepdim=True)
    if ignore_index is not None:
        pad_mask = target.eq(ignore_index)
        nll_loss.masked_fill_(pad_mask, 0.0)
        smooth_loss.masked_fill_(pad_mask, 0.0)
    nll_loss, smooth_loss = nll_loss.squeeze(-1), smooth_loss.squeeze(-1)
    if reduce:
        nll_loss, smooth_loss = nll_loss.sum(), smooth_loss.sum()
    eps_i = epsilon / (lprobs.size(-1) - 1)
    loss = (1.0 - epsilon - eps_i) * nll_loss + eps_i * smooth_loss
    return loss, nll_loss


def build(preexisting_criteria=("speech_to_unit",)):
    """-> {module name: module} for sys.modules, plus the registries under "_regs"."""
    regs = {"task": {}, "model": {}, "arch": {}, "arch_cfg": {}, "criterion": {}}

    def deco(kind, *_, **__):
        def reg(name, **kw):
            def d(cls):
                assert name not in regs[kind], f"duplicate {kind} {name}"
                regs[kind][name] = cls
                return cls
            return d
        return reg

    # ------------------------------------------------------------------ data
    class FairseqDataset(torch.utils.data.Dataset):
        def ordered_indices(self):
            return np.arange(len(self), dtype=np.int64)

        def set_epoch(self, epoch):
            pass

        def filter_indices_by_size(self, indices, max_sizes):
            keep = [i for i in indices if all(s <= m for s, m in zip(np.atleast_1d(self.size(i)),
                                                                      np.atleast_1d(max_sizes)) if m is not None)]
            ignored = [i for i in indices if i not in set(keep)]
            return np.asarray(keep, dtype=np.int64), ignored

        def batch_by_size(self, indices, max_tokens=None, max_sentences=None, required_batch_size_multiple=1):
            """data_utils.batch_by_size: walk the indices, close a batch when adding one more
            sample would exceed max_tokens (num_tokens = max sample size * batch size) or
            max_sentences; the closed batch keeps a multiple of required_batch_size_multiple."""
            batches, cur, cur_max = [], [], 0
            mult = required_batch_size_multiple
            for i in indices:
                n = self.num_tokens(int(i))
                new_max = max(cur_max, n)
                full = (max_tokens is not None and (len(cur) + 1) * new_max > max_tokens) or \
                       (max_sentences is not None and len(cur) == max_sentences)
                if cur and full:
                    keep = max(mult * (len(cur) // mult), len(cur) % mult)
                    batches.append(cur[:keep])
                    cur = cur[keep:]
                    cur_max = max((self.num_tokens(j) for j in cur), default=0)
                    new_max = max(cur_max, n)
                cur.append(int(i))
                cur_max = new_max
            if cur:
                batches.append(cur)
            return batches

    # ------------------------------------------------------------------ models
    class BaseFairseqModel(torch.nn.Module):
        def set_num_updates(self, num_updates):
            self.num_updates = num_updates

        def load_state_dict(self, state_dict, strict=True, model_cfg=None, args=None):
            return super().load_state_dict(state_dict, strict)

    class FairseqEncoderModel(BaseFairseqModel):
        def __init__(self, encoder):
            super().__init__()
            self.encoder = encoder

        def forward(self, src_tokens, src_lengths=None, **kw):
            return self.encoder(src_tokens, src_lengths, **kw)

        def get_normalized_probs(self, net_output, log_probs, sample=None):
            logits = net_output["encoder_out"].float()
            return F.log_softmax(logits, dim=-1) if log_probs else F.softmax(logits, dim=-1)

    class FairseqMultiModel(BaseFairseqModel):
        def __init__(self, decoder):
            super().__init__()
            self.decoder = decoder

    class CTCDecoder(torch.nn.Module):
        """fairseq.models.speech_to_speech.modules.ctc_decoder.CTCDecoder."""

        def __init__(self, dictionary, in_dim):
            super().__init__()
            self.dictionary = dictionary
            self.proj = torch.nn.Linear(in_dim, len(dictionary))

        def forward(self, src_tokens, src_lengths=None, **kw):
            return {"encoder_out": self.proj(src_tokens)}

    class S2STransformerMultitaskModelBase:
        @classmethod
        def build_multitask_decoder(cls, args, tgt_dict, in_dim):
            if args.decoder_type != "ctc":
                raise NotImplementedError("stub: ctc multitask decoders only")
            return CTCDecoder(dictionary=tgt_dict, in_dim=in_dim)

    def build_model(args, task, from_checkpoint=False):
        regs["arch_cfg"][args.arch](args)
        return regs["arch"][args.arch].build_model(args, task)

    def register_model_architecture(model_name, arch_name):
        def d(fn):
            regs["arch"][arch_name] = regs["model"][model_name]
            regs["arch_cfg"][arch_name] = fn
            return fn
        return d

    # ------------------------------------------------------------------ criteria
    class FairseqCriterion(torch.nn.Module):
        def __init__(self, task):
            super().__init__()
            self.task = task
            td = getattr(task, "target_dictionary", None)
            self.padding_idx = td.pad() if td is not None else -100

        @classmethod
        def build_criterion(cls, args, task):
            """FairseqCriterion.build_criterion: __init__ arguments filled from args by name."""
            kw = {}
            for p in inspect.signature(cls).parameters.values():
                if p.name == "task":
                    kw["task"] = task
                elif hasattr(args, p.name):
                    kw[p.name] = getattr(args, p.name)
                elif p.default is inspect.Parameter.empty:
                    raise NotImplementedError(f"unable to infer Criterion argument {p.name}")
            return cls(**kw)

    class CtcCriterion(FairseqCriterion):
        """fairseq.criterions.ctc.CtcCriterion (blank <s> = 0, reduction sum)."""

        def __init__(self, task, zero_infinity=True):
            super().__init__(task)
            self.blank_idx = 0
            self.pad_idx, self.eos_idx = task.target_dictionary.pad(), task.target_dictionary.eos()
            self.zero_infinity = zero_infinity

        def forward(self, model, sample, reduce=True, **kw):
            net_output = model(**sample["net_input"])
            lprobs = model.get_normalized_probs(net_output, log_probs=True).contiguous()
            input_lengths = sample["net_input"]["src_lengths"]
            pad_mask = (sample["target"] != self.pad_idx) & (sample["target"] != self.eos_idx)
            targets_flat = sample["target"].masked_select(pad_mask)
            target_lengths = sample["target_lengths"] if "target_lengths" in sample else pad_mask.sum(-1)
            loss = F.ctc_loss(lprobs, targets_flat, input_lengths, target_lengths, blank=self.blank_idx,
                              reduction="sum", zero_infinity=self.zero_infinity)
            return loss, sample["ntokens"], {"loss": loss.detach()}

    class SpeechToUnit(FairseqCriterion):
        """fairseq speech_to_unit = the reference's criterion (speech_to_speech_criterion.py:39-102)
        with rdrop_alpha 0, report_accuracy False."""

        def __init__(self, task, sentence_avg=False, label_smoothing=0.0, ignore_prefix_size=0):
            super().__init__(task)
            self.sentence_avg, self.eps, self.ignore_prefix_size = sentence_avg, label_smoothing, ignore_prefix_size
            # MultitaskCriterion.__init__(task.multitask_tasks, rdrop_alpha)
            self.multitask_criterion, self.multitask_loss_weight = {}, {}
            for name, t in task.multitask_tasks.items():
                if t.args.decoder_type != "ctc":
                    raise NotImplementedError("stub: ctc multitask criteria only")
                self.multitask_loss_weight[name] = t.args.loss_weight
                self.multitask_criterion[name] = CtcCriterion(t, t.args.zero_infinity)

        def forward(self, model, sample, reduce=True):
            net_input_concat = {
                "src_tokens": sample["net_input"]["src_tokens"],
                "src_lengths": sample["net_input"]["src_lengths"],
                "prev_output_tokens": sample["net_input"]["prev_output_tokens"],
                "tgt_speaker": sample["net_input"].get("tgt_speaker", None),
                "return_all_hiddens": True,
            }
            for item in sample["net_input"]:
                if item not in net_input_concat:
                    net_input_concat[item] = sample["net_input"][item]
            net_output, extra = model(**net_input_concat)
            loss, nll_loss = self.compute_loss(model, [net_output], sample, reduce=reduce)
            sample_size = sample["target"].size(0) if self.sentence_avg else sample["ntokens"]
            logging_output = {"loss": loss.data, "nll_loss": nll_loss.data, "ntokens": sample["ntokens"],
                              "nsentences": sample["target"].size(0), "sample_size": sample_size}
            if len(self.multitask_criterion) == 0:
                return loss, sample_size, logging_output
            multitask_loss, multitask_log = self.get_multitask_loss(model, sample, extra)
            loss += multitask_loss
            logging_output["multitask"] = multitask_log
            return loss, sample_size, logging_output

        def compute_loss(self, model, net_output, sample, reduce=True):
            lprobs = model.get_normalized_probs(net_output, log_probs=True)
            target = model.get_targets(sample, net_output)
            if self.ignore_prefix_size > 0:
                lprobs, target = lprobs[:, self.ignore_prefix_size:, :], target[:, self.ignore_prefix_size:]
            return _label_smoothed_nll_loss(lprobs.view(-1, lprobs.size(-1)), target.view(-1), self.eps,
                                            ignore_index=self.padding_idx, reduce=reduce)

        def get_multitask_loss(self, model, sample, model_out):
            loss, log = 0.0, {}
            for name, crit in self.multitask_criterion.items():
                layer_id = crit.task.args.input_layer
                if crit.task.args.input_from != "encoder":
                    raise NotImplementedError("stub: encoder-state multitask heads only")
                states = model_out["encoder_states"][layer_id]
                if len(model_out["encoder_padding_mask"]) > 0:
                    non_padding_mask = ~model_out["encoder_padding_mask"][0]
                else:
                    non_padding_mask = states.new_ones(states.size(1), states.size(0)).bool()
                task_sample = {"net_input": {"src_tokens": states, "src_lengths": non_padding_mask.long().sum(-1)},
                               "id": sample["id"]}
                for key in ("target", "target_lengths", "ntokens"):
                    task_sample[key] = sample["multitask"][name][key]
                task_loss, _, task_log = crit(model.multitask_decoders[name], task_sample)
                loss = loss + self.multitask_loss_weight[name] * task_loss
                log[name] = task_log
            return loss, log

        @staticmethod
        def logging_outputs_can_be_summed():
            return False

    def build_criterion(args, task):
        return regs["criterion"][args.criterion].build_criterion(args, task)

    for c in preexisting_criteria:
        regs["criterion"][c] = SpeechToUnit

    # ------------------------------------------------------------------ tasks
    class LegacyFairseqTask:
        def __init__(self, args):
            self.args = args
            self.datasets = {}

        @classmethod
        def setup_task(cls, args, **kw):
            return cls(args)

        def load_dataset(self, split, combine=False, **kw):
            raise NotImplementedError

        @property
        def source_dictionary(self):
            raise NotImplementedError

        @property
        def target_dictionary(self):
            raise NotImplementedError

        def dataset(self, split):
            if split not in self.datasets:
                raise KeyError("Dataset not loaded: " + split)
            return self.datasets[split]

        def build_model(self, args, from_checkpoint=False):
            return build_model(args, self, from_checkpoint)

        def build_criterion(self, args):
            return build_criterion(args, self)

        def max_positions(self):
            return None

        def get_batch_iterator(self, dataset, max_tokens=None, max_sentences=None, max_positions=None,
                               ignore_invalid_inputs=False, required_batch_size_multiple=1, seed=1,
                               num_shards=1, shard_id=0, epoch=1, **kw):
            dataset.set_epoch(epoch)
            indices = dataset.ordered_indices()
            if max_positions is not None:
                indices, ignored = dataset.filter_indices_by_size(indices, max_positions)
                if ignored and not ignore_invalid_inputs:
                    raise Exception(f"{len(ignored)} samples exceed max_positions")
            batches = dataset.batch_by_size(indices, max_tokens=max_tokens, max_sentences=max_sentences,
                                            required_batch_size_multiple=required_batch_size_multiple)
            return [dataset.collater([dataset[i] for i in b]) for b in batches[shard_id::num_shards]]

    def setup_task(args, **kw):
        return regs["task"][args.task].setup_task(args, **kw)

    # ------------------------------------------------------------------ multitask config
    class _Dict:
        """fairseq Dictionary over dict.txt (<s> <pad> </s> <unk> first)."""

        def __init__(self, path):
            self.symbols = ["<s>", "<pad>", "</s>", "<unk>"]
            with open(path, encoding="utf-8") as f:
                for line in f:
                    if line.strip():
                        tok = line.rstrip("\n").rsplit(" ", 1)[0]
                        if tok not in self.symbols:
                            self.symbols.append(tok)

        def __len__(self):
            return len(self.symbols)

        def pad(self):
            return 1

        def eos(self):
            return 2

    class SingleTaskConfig:
        def __init__(self, name, cfg):
            self.task_name, self.config = name, cfg
            self.tgt_dict = _Dict(cfg["dict"])
            self.decoder_type = cfg.get("decoder_type", "transformer")
            self.input_from = "decoder" if "decoder_layer" in cfg else "encoder"
            self.input_layer = int(cfg.get("decoder_layer" if self.input_from == "decoder" else "encoder_layer", 0)) - 1
            self.loss_weight = float(cfg.get("loss_weight", 0.0))
            self.zero_infinity = bool(cfg.get("zero_infinity", True))

    class MultitaskConfig:
        def __init__(self, path):
            import yaml
            with open(path) as f:
                self.config = {k: SingleTaskConfig(k, v or {}) for k, v in (yaml.safe_load(f) or {}).items()}
            self.first_pass_decoder_task_index = -1

        def get_all_tasks(self):
            return self.config

    class DummyMultiTask(LegacyFairseqTask):
        def __init__(self, args, tgt_dict, first_pass=False):
            super().__init__(args)
            self.tgt_dict, self.first_pass = tgt_dict, first_pass

        @property
        def target_dictionary(self):
            return self.tgt_dict

    # ------------------------------------------------------------------ utils
    def apply_to_sample(f, x):
        if torch.is_tensor(x):
            return f(x)
        if isinstance(x, dict):
            return {k: apply_to_sample(f, v) for k, v in x.items()}
        if isinstance(x, list):
            return [apply_to_sample(f, v) for v in x]
        if isinstance(x, tuple):
            return tuple(apply_to_sample(f, v) for v in x)
        return x

    def move_to_cuda(sample, device=None):
        return apply_to_sample(lambda t: t.to(device or "cuda", non_blocking=True), sample)

    def apply_half(sample):
        return apply_to_sample(lambda t: t.half() if t.dtype is torch.float32 else t, sample)

    # ------------------------------------------------------------------ modules
    mods = {}

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        mods[name] = m
        return m

    mod("fairseq")
    mod("fairseq.tasks", LegacyFairseqTask=LegacyFairseqTask, FairseqTask=LegacyFairseqTask, setup_task=setup_task,
        register_task=deco("task"), TASK_REGISTRY=regs["task"])
    mod("fairseq.tasks.speech_to_speech", DummyMultiTask=DummyMultiTask)
    mod("fairseq.data", FairseqDataset=FairseqDataset)
    mod("fairseq.data.audio")
    mod("fairseq.data.audio.data_cfg", MultitaskConfig=MultitaskConfig)
    mod("fairseq.models", BaseFairseqModel=BaseFairseqModel, FairseqEncoderModel=FairseqEncoderModel,
        FairseqMultiModel=FairseqMultiModel, register_model=deco("model"),
        register_model_architecture=register_model_architecture, build_model=build_model,
        MODEL_REGISTRY=regs["model"], ARCH_MODEL_REGISTRY=regs["arch"])
    mod("fairseq.models.speech_to_speech")
    mod("fairseq.models.speech_to_speech.s2s_transformer",
        S2STransformerMultitaskModelBase=S2STransformerMultitaskModelBase)
    mod("fairseq.criterions", FairseqCriterion=FairseqCriterion, register_criterion=deco("criterion"),
        CRITERION_REGISTRY=regs["criterion"], build_criterion=build_criterion)
    mod("fairseq.utils", move_to_cuda=move_to_cuda, apply_half=apply_half, apply_to_sample=apply_to_sample)
    for name, m in mods.items():
        parent, _, leaf = name.rpartition(".")
        if parent:
            setattr(mods[parent], leaf, m)
    mods["_regs"] = regs
    mods["_SpeechToUnit"] = SpeechToUnit
    return mods


def install(monkeypatch, **kw):
    """Put the stub into sys.modules (undone by monkeypatch) -> (fairseq module, registries)."""
    mods = build(**kw)
    for name, m in mods.items():
        if not name.startswith("_"):
            monkeypatch.setitem(sys.modules, name, m)
    return mods["fairseq"], mods["_regs"]


def train_args(parser_args):
    """Namespace with the fields fairseq's option parser would add for the canonical command."""
    a = Namespace(**vars(parser_args))
    a.sentence_avg = False
    a.ignore_prefix_size = 0
    return a


TINY = ("--encoder-layers 2 --decoder-layers 2 --encoder-embed-dim 256 --encoder-ffn-embed-dim 1024 "
        "--encoder-attention-heads 4 --decoder-attention-heads 4")


def dropin_setup(monkeypatch, tmp_path, fusion_yaml, multitask=False, extra=""):
    """Stub fairseq installed, a tiny on-disk corpus (tests/manifest_corpus.py) and the parsed
    canonical command for it (tiny dims) -> (fairseq module, registries, args, corpus, adapter
    registration result)."""
    from conftest import pkg
    from manifest_corpus import write_corpus
    fs, regs = install(monkeypatch)
    d = tmp_path / "data"
    d.mkdir()
    c = write_corpus(str(d), frames=(150, 97, 200, 61, 88, 131), di=768, ti=12)
    y = tmp_path / "mm.yaml"
    y.write_text(fusion_yaml.replace('["/feats/vit_base_patch16_384"]', f'["{c["feat_dir"]}"]'))
    mt_arg = ""
    if multitask:
        letters = "abcdefghij"
        mtd = tmp_path / "letters"
        mtd.mkdir()
        (mtd / "dict.txt").write_text("".join(f"{ch} 1\n" for ch in letters))
        rng = np.random.default_rng(0)
        rows = ["id\ttgt_text"] + [f"utt{k}\t{' '.join(rng.choice(list(letters), max(2, T // 20)))}"
                                   for k, T in enumerate(c["frames"])]
        (mtd / "train.tsv").write_text("\n".join(rows) + "\n")
        mt = tmp_path / "config_multitask.yaml"
        mt.write_text(f"target_ctc:\n  decoder_type: ctc\n  dict: {mtd}/dict.txt\n  data: {mtd}\n"
                      f"  encoder_layer: 1\n  loss_weight: 1.5\n")
        mt_arg = f" --multitask-config-yaml {mt}"
    argv = (f"{d} --task multimodal_speech_to_speech --arch mm_s2ut_transformer --criterion speech_to_unit "
            f"--config-yaml config.yaml --target-is-code --target-code-size 1000 --label-smoothing 0.2 "
            f"--share-decoder-input-output-embed --fp16 --multimodal-translation-config-yaml {y} {TINY}"
            f"{mt_arg} {extra}")
    args = train_args(pkg("plugins").build_parser().parse_args(argv.split()))
    reg = pkg("fairseq_adapter").register(fs)
    return fs, regs, args, c, reg
