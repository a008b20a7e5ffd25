"""Writes a small on-disk Speech-Multi30K-shaped corpus the way the reference's preprocessing lays
it out: ``{split}.tsv`` (id, src_audio, src_n_frames, tgt_text, tgt_n_frames),
16-bit mono 16 kHz WAVs named ``{image row + 1}.wav``, ``config.yaml`` (audio_root, transforms),
and image features ``{split}.pth`` [N, Ti, Di] fp32 + ``{split}_mask.pth`` [N, Ti] bool."""
import os

import numpy as np
import torch

from conftest import pkg
from oracle import ref_fbank as RF


def write_corpus(root, frames=(120, 57, 200, 57, 88), n_images=8, ti=9, di=16, seed=0, split="train",
                 transforms=("utterance_cmvn",), specaugment=None, with_mask=True):
    M = pkg("manifest")
    rng = np.random.default_rng(seed)
    wav_dir = os.path.join(root, "wav")
    os.makedirs(wav_dir, exist_ok=True)
    rows = rng.permutation(n_images)[: len(frames)]
    lines = ["id\tsrc_audio\tsrc_n_frames\ttgt_text\ttgt_n_frames"]
    waves, units = [], []
    for k, (T, row) in enumerate(zip(frames, rows)):
        w = np.round(RF.synth_wave(T, rng)).clip(-32768, 32767).astype(np.float32)
        name = f"{int(row) + 1}.wav"
        M.write_wav(os.path.join(wav_dir, name), w)
        u = rng.integers(0, 1000, max(1, int(round(0.3 * T))))
        units.append(u)
        waves.append(w)
        lines.append(f"utt{k}\t{name}\t{T}\t{' '.join(map(str, u))}\t{len(u)}")
    with open(os.path.join(root, f"{split}.tsv"), "w") as f:
        f.write("\n".join(lines) + "\n")
    cfg = [f"audio_root: {wav_dir}", "input_channels: 1", "input_feat_per_channel: 80", "transforms:",
           "  '*': [utterance_cmvn]", f"  _train: [{', '.join(transforms)}]"]
    if specaugment:
        cfg.append("specaugment:")
        cfg += [f"  {k}: {v}" for k, v in specaugment.items()]
    with open(os.path.join(root, "config.yaml"), "w") as f:
        f.write("\n".join(cfg) + "\n")
    feat_dir = os.path.join(root, "img")
    os.makedirs(feat_dir, exist_ok=True)
    feats = torch.from_numpy(rng.standard_normal((n_images, ti, di)).astype(np.float32))
    torch.save(feats, os.path.join(feat_dir, f"{split}.pth"))
    mask = None
    if with_mask:
        mask = torch.zeros(n_images, ti, dtype=torch.bool)
        for r in range(n_images):
            mask[r, int(rng.integers(ti // 2, ti + 1)):] = True
        torch.save(mask, os.path.join(feat_dir, f"{split}_mask.pth"))
    return {"waves": waves, "units": units, "rows": rows, "feats": feats, "mask": mask, "feat_dir": feat_dir,
            "frames": list(frames)}
