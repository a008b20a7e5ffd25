"""On-disk data path: TSV manifest + 16-bit WAV sources + unit targets +
pre-extracted image features -> collated batches whose fbank/CMVN run on the GPU.

What the reference does per utterance on the CPU, in DataLoader workers
(mm_s2ut/data/speech_to_speech_dataset.py):
  * ``MultiModalSpeechToSpeechDatasetCreator.from_tsv`` :658-703 / ``_from_list`` :557-655 —
    ``{root}/{split}.tsv`` with columns id, src_audio, src_n_frames, tgt_text (unit ids), tgt_n_frames;
    ``src_audio`` joined onto ``data_cfg.audio_root``; image features ``{feat_path}/{split}.pth``
    (+ optional ``{split}_mask.pth``) per ``image_feat_path`` entry (:606-616, ``ImageDataset`` :36-68).
  * ``get_source_audio`` :234-274 — ``sf.read(float32)`` then ``get_features_or_waveform`` ->
    ``get_fbank`` (audio_utils.py:326-349): mono, ×2^15, Kaldi fbank; then the data config's
    feature transforms (utterance CMVN).
  * ``__getitem__`` :276-342 — target = ``tgt_dict.encode_line(tgt_text, append_eos=True)``;
    image row = int(stem of the audio file name) - 1 (:319-320).
  * ``collater`` :377-471 (restated in ``data.collater``).

Here the host keeps only file IO (a prefetch thread reads the next batch's WAV files, targets and
image rows while the GPU trains on the current one); the waveforms go to HBM through pinned
memory and ``FbankFrontend`` turns them into the model's fp16 ``src_tokens`` in two launches
(fbank for every frame of the batch, CMVN + zero-padded collation).

The unit dictionary follows fairseq ``SpeechToSpeechTask.setup_task`` for ``--target-is-code``:
``Dictionary()`` (``<s>`` 0, ``<pad>`` 1, ``</s>`` 2, ``<unk>`` 3) plus the symbols "0" ..
str(target_code_size - 1), so unit u maps to id u + 4.
"""
import concurrent.futures
import csv
import os
import re
import wave

import numpy as np
import torch

from . import data as D
from .frontend import n_frames as fbank_frames

BOS, PAD, EOS, UNK = 0, 1, 2, 3
_SPACE = re.compile(r"\s+")


def load_samples_from_tsv(root, split):
    """fairseq ``SpeechToTextDatasetCreator._load_samples_from_tsv``: tab-separated, no quoting."""
    path = os.path.join(root, f"{split}.tsv")
    if not os.path.isfile(path):
        raise FileNotFoundError(f"Dataset not found: {path}")
    with open(path, newline="") as f:
        reader = csv.DictReader(f, delimiter="\t", quotechar=None, doublequote=False,
                                lineterminator="\n", quoting=csv.QUOTE_NONE)
        samples = [dict(e) for e in reader]
    if len(samples) == 0:
        raise ValueError(f"Empty manifest: {path}")
    return samples


class UnitDictionary:
    """The subset of fairseq ``Dictionary`` the unit targets use (specials first, then symbols)."""

    def __init__(self, symbols=()):
        self.symbols = ["<s>", "<pad>", "</s>", "<unk>"]
        self.indices = {s: i for i, s in enumerate(self.symbols)}
        for s in symbols:
            self.add_symbol(s)

    @classmethod
    def for_codes(cls, target_code_size):
        return cls(str(i) for i in range(target_code_size))

    def add_symbol(self, s):
        if s not in self.indices:
            self.indices[s] = len(self.symbols)
            self.symbols.append(s)
        return self.indices[s]

    def __len__(self):
        return len(self.symbols)

    def pad(self):
        return PAD

    def eos(self):
        return EOS

    def encode_line(self, line, append_eos=True):
        """fairseq ``Dictionary.encode_line`` with ``tokenize_line`` and add_if_not_exist=False."""
        words = _SPACE.sub(" ", line).strip().split()
        ids = [self.indices.get(w, UNK) for w in words]
        if append_eos:
            ids.append(EOS)
        return torch.tensor(ids, dtype=torch.long)


def read_wav(path):
    """16-bit PCM WAV -> (float32 samples in int16 range, sample rate): the reference's
    ``sf.read(dtype="float32")`` (x / 2^15) followed by ``get_waveform(normalization=False)``'s
    × 2^15, which round-trips int16 exactly.  Multi-channel input is averaged to mono (sox
    ``channels 1``, as fairseq ``convert_waveform(to_mono=True)``)."""
    with wave.open(path, "rb") as w:
        if w.getsampwidth() != 2:
            raise ValueError(f"{path}: only 16-bit PCM WAV is supported (got {8 * w.getsampwidth()}-bit)")
        ch, sr, n = w.getnchannels(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    x = np.frombuffer(raw, dtype="<i2").astype(np.float32)
    if ch > 1:
        x = x.reshape(-1, ch).mean(axis=1, dtype=np.float32)
    return x, sr


def write_wav(path, samples, sample_rate=16000):
    """int16-range float/int samples -> 16-bit mono PCM WAV (test / tooling helper)."""
    s = np.clip(np.round(np.asarray(samples, dtype=np.float64)), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sample_rate)
        w.writeframes(s.tobytes())


class ImageFeatures:
    """``ImageDataset`` (speech_to_speech_dataset.py:36-68) without raw-image paths:
    ``{split}.pth`` [N, Ti, Di] and optional ``{split}_mask.pth`` [N, Ti] bool, loaded with
    ``torch.load(weights_only=True)`` (tensors only; nothing in the file is executed)."""

    def __init__(self, feat_dir, split):
        fp = os.path.join(feat_dir, split + ".pth")
        if not os.path.exists(fp):
            raise FileNotFoundError(f"not found image feature: {fp}")
        self.feat = torch.load(fp, map_location="cpu", weights_only=True)
        mp = os.path.join(feat_dir, split + "_mask.pth")
        self.mask = torch.load(mp, map_location="cpu", weights_only=True) if os.path.exists(mp) else None
        if self.mask is not None and self.mask.shape[0] != self.feat.shape[0]:
            raise ValueError(f"{mp}: {self.mask.shape[0]} masks for {self.feat.shape[0]} features")

    def __len__(self):
        return self.feat.shape[0]

    def __getitem__(self, row):
        return self.feat[row], (None if self.mask is None else self.mask[row].to(torch.bool))


def load_data_config(path):
    """The parts of fairseq ``S2SDataConfig`` (config.yaml) the path reads: audio_root,
    input_feat_per_channel, and the feature transforms (utterance_cmvn is the one built)."""
    cfg = {"audio_root": "", "input_feat_per_channel": 80, "transforms": {}}
    if path is not None and os.path.exists(path):
        import yaml
        with open(path) as f:
            cfg.update(yaml.safe_load(f) or {})
    return cfg


def feature_transforms(data_cfg, split, is_train):
    """fairseq ``S2TDataConfig.get_transforms``: the split's own list, else ``_train`` for a
    training split, else ``*``."""
    t = data_cfg.get("transforms") or {}
    names = t.get(split)
    if names is None and is_train:
        names = t.get("_train")
    if names is None:
        names = t.get("*")
    return list(names or [])


class MultiModalS2SManifest:
    """One split of the on-disk corpus (``MultiModalSpeechToSpeechDatasetCreator._from_list``)."""

    def __init__(self, root, split, tgt_dict, data_cfg=None, image_feat_path=None, is_train=None,
                 max_source_positions=6000, max_target_positions=1024, multitask=None):
        """multitask: {task: (raw config, multitask.Dictionary)} (--multitask-config-yaml): each
        task's text targets (``{data}/{split}.tsv``) join every collated batch as
        sample["multitask"] (speech_to_speech_dataset.py:474-521)."""
        self.root, self.split = root, split
        self.multitask = {}
        if multitask:
            from . import multitask as MT
            for name, (raw, dct) in multitask.items():
                self.multitask[name] = MT.TextTargetMultitaskData(raw["data"], split, dct,
                                                                   raw.get("decoder_type", "transformer"))
        self.data_cfg = data_cfg or load_data_config(os.path.join(root, "config.yaml"))
        self.is_train = split.startswith("train") if is_train is None else is_train
        samples = load_samples_from_tsv(root, split)
        audio_root = self.data_cfg.get("audio_root") or ""
        self.ids = [s["id"] for s in samples]
        self.audio_paths = [os.path.join(audio_root, s["src_audio"]) for s in samples]
        self.n_frames = np.array([int(s["src_n_frames"]) for s in samples], dtype=np.int64)
        self.tgt_texts = [s["tgt_text"] for s in samples]
        self.tgt_n_frames = np.array([int(s["tgt_n_frames"]) for s in samples], dtype=np.int64)
        self.tgt_dict = tgt_dict
        self.images = None
        if image_feat_path:
            paths = [image_feat_path] if isinstance(image_feat_path, str) else list(image_feat_path)
            if len(paths) != 1:
                raise NotImplementedError("one image-feature type (SURVEY Q8)")
            self.images = ImageFeatures(paths[0], split)
        tf = feature_transforms(self.data_cfg, split, self.is_train)
        unknown = [t for t in tf if t not in ("utterance_cmvn", "specaugment")]
        if unknown:
            raise NotImplementedError(f"feature transforms {unknown} (utterance_cmvn, specaugment are built)")
        if "specaugment" in tf and "utterance_cmvn" in tf and tf.index("specaugment") < tf.index("utterance_cmvn"):
            raise NotImplementedError("specaugment before utterance_cmvn (the GPU path masks after CMVN)")
        self.cmvn = "utterance_cmvn" in tf
        self.specaugment = None
        if "specaugment" in tf:
            from .frontend import SpecAugment
            self.specaugment = SpecAugment.from_config_dict(self.data_cfg.get("specaugment"))
        self.max_source_positions = max_source_positions
        self.max_target_positions = max_target_positions

    def __len__(self):
        return len(self.ids)

    def image_row(self, i):
        """speech_to_speech_dataset.py:319-320: the audio file's stem is the 1-based image row."""
        stem = os.path.splitext(os.path.basename(self.audio_paths[i]))[0]
        return int(stem) - 1

    def item(self, i):
        wav, sr = read_wav(self.audio_paths[i])
        if sr != 16000:
            raise ValueError(f"{self.audio_paths[i]}: {sr} Hz (the fbank front end is 16 kHz)")
        it = {"index": i, "audio_path": self.audio_paths[i], "wave": wav,
              "n_frames": fbank_frames(len(wav)),
              "target": self.tgt_dict.encode_line(self.tgt_texts[i], append_eos=True)}
        if self.images is not None:
            img, m = self.images[self.image_row(i)]
            it["img"] = img
            if m is not None:
                it["img_mask"] = m
        return it

    def ordered_indices(self, seed=1, epoch=1):
        """``SpeechToTextDataset.ordered_indices``: longest first; ties shuffled for train."""
        if self.is_train:
            tie = np.random.RandomState((seed + epoch) % 2 ** 32).permutation(len(self))
        else:
            tie = np.arange(len(self))
        return np.lexsort([tie, -self.n_frames])

    def batches(self, max_tokens=40000, seed=1, epoch=1, skip_invalid=False):
        """fairseq ``filter_indices_by_size`` (src frames vs max_source_positions, target tokens
        vs max_target_positions) then ``batch_by_size`` over the ordered indices."""
        order = self.ordered_indices(seed, epoch)
        ok = (self.n_frames[order] <= self.max_source_positions) & \
             (self.tgt_n_frames[order] + 1 <= self.max_target_positions) & \
             (self.n_frames[order] <= max_tokens)
        if not ok.all():
            if not skip_invalid:
                bad = order[~ok][:10].tolist()
                raise ValueError(f"{int((~ok).sum())} samples exceed the size limits (first ids {bad}); "
                                 "pass skip_invalid=True (--skip-invalid-size-inputs-valid-test)")
            order = order[ok]
        return D.batch_by_size(self.n_frames, max_tokens, order=order)

    def collate(self, indices):
        """Host half of a batch: items read from disk, collated in the reference's order; the
        waveforms are returned in that same (length-descending) order for the GPU front end."""
        items = [self.item(int(i)) for i in indices]
        for it in items:
            if it["n_frames"] <= 0:
                raise ValueError(f"{it['audio_path']}: shorter than one 25 ms frame")
        sample = D.collater(items)
        by_index = {it["index"]: it for it in items}
        waves = [by_index[int(i)]["wave"] for i in sample["id"].tolist()]
        if self.multitask:
            from . import multitask as MT
            pos = {int(i): k for k, i in enumerate(indices)}
            order = torch.tensor([pos[int(i)] for i in sample["id"].tolist()], dtype=torch.long)
            sample["multitask"] = MT.sample_multitask(
                {n: (d, [d.get(self.ids[int(i)]) for i in indices]) for n, d in self.multitask.items()}, order)
        return sample, waves


class DeviceLoader:
    """Batches of a manifest split, resident on ``device``: a one-deep prefetch thread does the
    file IO and collation of batch i+1 while batch i trains; waveforms are copied from pinned
    memory and turned into fp16 ``src_tokens`` by the GPU front end.  Yields DeviceBatch objects
    (``runtime.prepare_batch``) plus the host sample."""

    def __init__(self, dataset, batches, cfg, device="cuda", frontend=None, prefetch=True, seed=1, epoch=1):
        from . import frontend as fe_mod
        self.ds, self.batches, self.cfg = dataset, list(batches), cfg
        self.device = torch.device(device)
        self.fe = frontend or fe_mod.FbankFrontend(self.device, cmvn=dataset.cmvn,
                                                   specaugment=dataset.specaugment)
        self.seed, self.epoch = seed, epoch
        self.pool = concurrent.futures.ThreadPoolExecutor(1) if prefetch else None

    def _host(self, b):
        sample, waves = self.ds.collate(self.batches[b])
        return sample, waves

    def _to_device(self, b, sample, waves):
        from . import runtime
        wb = self.fe.upload(waves, pin=True)
        if wb["order"] != list(range(len(waves))):
            raise AssertionError("front-end order differs from the collater's")
        rng = np.random.RandomState((self.seed * 1000003 + self.epoch * 7919 + b) % 2 ** 32) \
            if self.fe.specaugment is not None else None
        src = self.fe(wb, rng)
        return runtime.prepare_batch(sample, self.cfg, self.device, src_override=src)

    def __iter__(self):
        n = len(self.batches)
        if self.pool is None:
            for b in range(n):
                sample, waves = self._host(b)
                yield self._to_device(b, sample, waves), sample
            return
        fut = self.pool.submit(self._host, 0) if n else None
        for b in range(n):
            sample, waves = fut.result()
            if b + 1 < n:
                fut = self.pool.submit(self._host, b + 1)
            yield self._to_device(b, sample, waves), sample

    def __len__(self):
        return len(self.batches)
