"""GPU fbank front end: waveforms resident in HBM -> 80-bin Kaldi log-mel -> utterance CMVN ->
zero-padded fp16 [B, Tmax, 80] (the model's src_tokens).

Moves the reference's per-utterance CPU feature extraction (speech_to_speech_dataset.py:234-274 ->
audio_utils.py:326-349 -> torchaudio.compliance.kaldi.fbank, then the data-config
utterance_cmvn transform and _collate_frames) onto the GPU: one launch for all frames of a batch,
one for CMVN + collation.
"""
import math

import numpy as np
import torch

from . import kernels as K

WIN, SHIFT, NFFT = 400, 160, 512


def mel_banks(num_bins=80, padded=NFFT, sample_freq=16000.0, low_freq=20.0, high_freq=0.0):
    """Triangular mel filters exactly as torchaudio.compliance.kaldi.get_mel_banks (vtln off),
    fp32, padded with a zero Nyquist column -> [num_bins, padded//2 + 1]."""
    nyq = 0.5 * sample_freq
    if high_freq <= 0.0:
        high_freq += nyq
    width = sample_freq / padded
    mlo = 1127.0 * math.log(1.0 + low_freq / 700.0)
    mhi = 1127.0 * math.log(1.0 + high_freq / 700.0)
    delta = (mhi - mlo) / (num_bins + 1)
    b = np.arange(num_bins, dtype=np.float32)[:, None]
    left = np.float32(mlo) + b * np.float32(delta)
    center = np.float32(mlo) + (b + 1.0) * np.float32(delta)
    right = np.float32(mlo) + (b + 2.0) * np.float32(delta)
    f = np.float32(width) * np.arange(padded // 2, dtype=np.float32)
    mel = (np.float32(1127.0) * np.log1p(f / np.float32(700.0)).astype(np.float32))[None, :]
    up = (mel - left) / (center - left)
    down = (right - mel) / (right - center)
    banks = np.maximum(np.float32(0.0), np.minimum(up, down)).astype(np.float32)
    return np.pad(banks, ((0, 0), (0, 1)))


def n_frames(n_samples):
    return 0 if n_samples < WIN else 1 + (n_samples - WIN) // SHIFT


class FbankFrontend:
    def __init__(self, device="cuda", num_bins=80, cmvn=True):
        self.device = torch.device(device)
        self.num_bins = num_bins
        self.cmvn = cmvn
        banks = mel_banks(num_bins)
        self.banks = torch.from_numpy(banks).to(self.device)
        nz = banks > 0
        lo = nz.argmax(1)
        hi = banks.shape[1] - nz[:, ::-1].argmax(1)
        lo[~nz.any(1)] = hi[~nz.any(1)] = 0
        rng = np.stack([lo, hi], 1).astype(np.int32)
        self.mel_range = torch.from_numpy(rng.reshape(-1)).to(self.device)

    def upload(self, waves):
        """waves: list of 1-D float32 arrays already in int16 range (get_waveform(normalization=False)).
        Returns a device-resident wave batch (sorted by frames, descending, like the collater)."""
        lens = [n_frames(len(w)) for w in waves]
        order = sorted(range(len(waves)), key=lambda i: -lens[i])
        waves = [waves[i] for i in order]
        fr = np.array([lens[i] for i in order], dtype=np.int64)
        wl = np.array([len(w) for w in waves], dtype=np.int64)
        wave_off = np.concatenate([[0], np.cumsum(wl)]).astype(np.int64)
        frame_off = np.concatenate([[0], np.cumsum(fr)]).astype(np.int32)
        flat = np.concatenate(waves).astype(np.float32)
        return {
            "wave": torch.from_numpy(flat).to(self.device),
            "wave_off": torch.from_numpy(wave_off).to(self.device),
            "frame_off": torch.from_numpy(frame_off).to(self.device),
            "n_frames": torch.from_numpy(fr), "total": int(fr.sum()), "Tmax": int(fr.max()),
            "B": len(waves), "order": order,
        }

    def __call__(self, wb):
        feats = K.fbank(wb["wave"], wb["wave_off"], wb["frame_off"], wb["total"], self.banks, self.mel_range,
                        self.num_bins)
        return K.cmvn_collate(feats, wb["frame_off"], wb["B"], wb["Tmax"], self.num_bins, self.cmvn)

    def features_f32(self, wb):
        """Raw log-mel features [total_frames, nbins] fp32 (no CMVN) — for parity tests."""
        return K.fbank(wb["wave"], wb["wave_off"], wb["frame_off"], wb["total"], self.banks, self.mel_range,
                       self.num_bins)
