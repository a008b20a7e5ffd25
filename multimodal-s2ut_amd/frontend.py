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


class SpecAugment:
    """fairseq ``SpecAugmentTransform`` (data/audio/feature_transforms/specaugment.py) parameters
    and its per-utterance mask draws; the masking itself runs on the GPU
    (``mms2ut_specaugment_f16``).  Draw order per utterance is the transform's: freq_mask_N ×
    (f ~ U[0, F), f0 ~ U[0, nbins - f)), then, if max_t = min(T_mask, floor(T·p)) >= 1,
    time_mask_N × (t ~ U[0, max_t), t0 ~ U[0, T - t)); a zero width masks nothing.  The draws use
    a seeded numpy stream per batch (the reference's global np.random in DataLoader workers is not
    replayable, so mask positions are not bit-matched to it)."""

    def __init__(self, time_warp_W=0, freq_mask_N=0, freq_mask_F=0, time_mask_N=0, time_mask_T=0,
                 time_mask_p=0.0, mask_value=None):
        if time_warp_W:
            raise NotImplementedError("SpecAugment time warping (time_warp_W > 0) is not built")
        self.fn, self.ff = int(freq_mask_N), int(freq_mask_F)
        self.tn, self.tt, self.tp = int(time_mask_N), int(time_mask_T), float(time_mask_p)
        self.mask_value = mask_value

    @classmethod
    def from_config_dict(cls, d):
        d = d or {}
        return cls(d.get("time_warp_W", 0), d.get("freq_mask_N", 0), d.get("freq_mask_F", 0),
                   d.get("time_mask_N", 0), d.get("time_mask_T", 0), d.get("time_mask_p", 0.0),
                   d.get("mask_value", None))

    def draws(self, n_frames, nbins, rng):
        """int32 [B, 2*(freq_mask_N + time_mask_N)] of (start, width) pairs."""
        out = np.zeros((len(n_frames), 2 * (self.fn + self.tn)), dtype=np.int32)
        for b, T in enumerate(n_frames):
            T = int(T)
            for k in range(self.fn):
                f = int(rng.randint(0, self.ff)) if self.ff > 0 else 0
                out[b, 2 * k: 2 * k + 2] = (int(rng.randint(0, nbins - f)), f)
            max_t = min(self.tt, math.floor(T * self.tp))
            if max_t < 1:
                continue
            for k in range(self.tn):
                t = int(rng.randint(0, max_t))
                j = 2 * (self.fn + k)
                out[b, j: j + 2] = (int(rng.randint(0, T - t)), t)
        return out


_FRONTENDS = {}


def wave_net_input_src(ni, device):
    """fp16 [B, Tmax, 80] src_tokens for a sample whose net_input carries waveforms instead of
    features (the fairseq-train drop-in's collater, fairseq_adapter.py): ``src_waves`` int32 [N]
    = the fp32 samples' bit patterns (so fairseq's apply_half leaves them alone), ``src_wave_offsets``
    int64 [B + 1], ``src_cmvn`` bool, optional ``src_specaugment`` {masks int32 [B, 2(nf + nt)],
    n_freq, n_time, mask_value} drawn by the collater (CPU worker, as the reference's transform)."""
    dev = torch.device(device)
    cmvn = bool(ni.get("src_cmvn", True))
    fe = _FRONTENDS.get((dev, cmvn))
    if fe is None:
        fe = _FRONTENDS[(dev, cmvn)] = FbankFrontend(dev, cmvn=cmvn)
    w = ni["src_waves"]
    if w.dtype != torch.int32:
        raise TypeError(f"src_waves: int32 bit patterns of fp32 samples expected, got {w.dtype}")
    wb = fe.from_device(w.to(dev).view(torch.float32), ni["src_wave_offsets"])
    feats = K.fbank(wb["wave"], wb["wave_off"], wb["frame_off"], wb["total"], fe.banks, fe.mel_range, fe.num_bins)
    out = K.cmvn_collate(feats, wb["frame_off"], wb["B"], wb["Tmax"], fe.num_bins, cmvn)
    sa = ni.get("src_specaugment")
    if sa is not None and sa["n_freq"] + sa["n_time"] > 0:
        K.specaugment(out, wb["frame_off"], sa["masks"].to(dev, torch.int32).contiguous(), int(sa["n_freq"]),
                      int(sa["n_time"]), sa.get("mask_value"))
    return out


class FbankFrontend:
    def __init__(self, device="cuda", num_bins=80, cmvn=True, specaugment=None):
        self.device = torch.device(device)
        self.num_bins = num_bins
        self.cmvn = cmvn
        self.specaugment = specaugment
        banks = mel_banks(num_bins)
        self.banks = torch.from_numpy(banks).to(self.device)
        nz = banks > 0
        lo = nz.argmax(1)
        hi = banks.shape[1] - nz[:, ::-1].argmax(1)
        lo[~nz.any(1)] = hi[~nz.any(1)] = 0
        rng = np.stack([lo, hi], 1).astype(np.int32)
        if int((hi - lo).sum()) > 1024:
            raise ValueError("fbank: more than 1024 nonzero mel weights (include/mms2ut.h mms2ut_fbank_f32)")
        self.mel_range = torch.from_numpy(rng.reshape(-1)).to(self.device)

    def upload(self, waves, pin=False):
        """waves: list of 1-D float32 arrays already in int16 range (get_waveform(normalization=False)).
        Returns a device-resident wave batch (sorted by frames, descending, like the collater).
        pin=True stages the samples in pinned host memory and copies asynchronously."""
        lens = [n_frames(len(w)) for w in waves]
        order = sorted(range(len(waves)), key=lambda i: -lens[i])
        waves = [waves[i] for i in order]
        fr = np.array([lens[i] for i in order], dtype=np.int64)
        wl = np.array([len(w) for w in waves], dtype=np.int64)
        wave_off = np.concatenate([[0], np.cumsum(wl)]).astype(np.int64)
        frame_off = np.concatenate([[0], np.cumsum(fr)]).astype(np.int32)
        flat = np.concatenate(waves).astype(np.float32)
        def dev(a):
            t = torch.from_numpy(a)
            return t.pin_memory().to(self.device, non_blocking=True) if pin else t.to(self.device)

        return {
            "wave": dev(flat), "wave_off": dev(wave_off), "frame_off": dev(frame_off),
            "n_frames": torch.from_numpy(fr), "total": int(fr.sum()), "Tmax": int(fr.max()),
            "B": len(waves), "order": order,
        }

    def __call__(self, wb, rng=None):
        """-> fp16 [B, Tmax, nbins].  With a SpecAugment policy and a numpy RandomState ``rng``
        (training batches), the masks are drawn on the host and applied in place after CMVN."""
        feats = K.fbank(wb["wave"], wb["wave_off"], wb["frame_off"], wb["total"], self.banks, self.mel_range,
                        self.num_bins)
        out = K.cmvn_collate(feats, wb["frame_off"], wb["B"], wb["Tmax"], self.num_bins, self.cmvn)
        sa = self.specaugment
        if sa is not None and rng is not None and sa.fn + sa.tn > 0:
            m = sa.draws(wb["n_frames"].tolist(), self.num_bins, rng)
            masks = torch.from_numpy(m).pin_memory().to(self.device, non_blocking=True)
            K.specaugment(out, wb["frame_off"], masks, sa.fn, sa.tn, sa.mask_value)
        return out

    def from_device(self, waves, wave_off):
        """A wave batch from samples already in HBM: ``waves`` fp32 [N] (utterances back to back, in
        the collater's frame-descending order), ``wave_off`` int64 [B + 1] sample offsets."""
        off = wave_off.cpu().numpy().astype(np.int64)
        fr = np.array([n_frames(int(n)) for n in np.diff(off)], dtype=np.int64)
        if len(fr) == 0 or np.any(fr <= 0) or np.any(np.diff(fr) > 0):
            raise ValueError(f"wave batch: frames {fr.tolist()} (need >= 1 frame each, descending order)")
        frame_off = np.concatenate([[0], np.cumsum(fr)]).astype(np.int32)
        return {"wave": waves.contiguous(), "wave_off": wave_off.to(self.device, torch.int64).contiguous(),
                "frame_off": torch.from_numpy(frame_off).to(self.device), "n_frames": torch.from_numpy(fr),
                "total": int(fr.sum()), "Tmax": int(fr.max()), "B": len(fr), "order": list(range(len(fr)))}

    def features_f32(self, wb):
        """Raw log-mel features [total_frames, nbins] fp32 (no CMVN) — for parity tests."""
        return K.fbank(wb["wave"], wb["wave_off"], wb["frame_off"], wb["total"], self.banks, self.mel_range,
                       self.num_bins)
