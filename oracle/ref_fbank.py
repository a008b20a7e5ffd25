"""numpy restatement of the reference's fbank front end — TEST INFRASTRUCTURE ONLY.

Path followed: ``get_source_audio`` (mm_s2ut/data/speech_to_speech_dataset.py:234-274) ->
``get_features_or_waveform`` (mm_s2ut/data/audio_utils.py:352-384) -> ``get_fbank``
(audio_utils.py:326-349) -> ``get_waveform(normalization=False)`` (×2^15, audio_utils.py:289-290)
-> fairseq ``_get_torchaudio_fbank`` -> ``torchaudio.compliance.kaldi.fbank(num_mel_bins=80)``
with its defaults (dither 0, snip_edges, round_to_power_of_two, povey window, preemphasis 0.97,
remove_dc_offset, low_freq 20, high_freq = Nyquist, use_power, use_log_fbank, eps = FLT_EPSILON,
no energy).  torchaudio is absent from the container (unpinned version) — the restatement is
cross-checked against transformers.audio_utils' independent Kaldi-compatible implementation.
Then the data-config ``utterance_cmvn`` transform (fairseq UtteranceCMVN; speech_to_speech_dataset.py:271-272)
and, for training splits whose config lists it, ``specaugment`` (fairseq SpecAugmentTransform).
"""
import numpy as np

FLT_EPS = np.float32(np.finfo(np.float32).eps)


def mel_scale(f):
    return 1127.0 * np.log(1.0 + f / 700.0)


def mel_banks(num_bins=80, padded=512, sample_freq=16000.0, low_freq=20.0, high_freq=0.0):
    """torchaudio.compliance.kaldi.get_mel_banks (vtln_warp=1), float32 -> [num_bins, padded//2]."""
    num_fft_bins = padded // 2
    nyquist = 0.5 * sample_freq
    if high_freq <= 0.0:
        high_freq += nyquist
    fft_bin_width = sample_freq / padded
    mel_low = mel_scale(low_freq)
    mel_high = mel_scale(high_freq)
    delta = (mel_high - mel_low) / (num_bins + 1)
    b = np.arange(num_bins, dtype=np.float32)[:, None]
    left = np.float32(mel_low) + b * np.float32(delta)
    center = np.float32(mel_low) + (b + 1.0) * np.float32(delta)
    right = np.float32(mel_low) + (b + 2.0) * np.float32(delta)
    mel = (np.float32(1127.0) * np.log1p(
        (np.float32(fft_bin_width) * np.arange(num_fft_bins, dtype=np.float32)) / np.float32(700.0)
    ).astype(np.float32))[None, :]
    up = (mel - left) / (center - left)
    down = (right - mel) / (right - center)
    return np.maximum(np.float32(0.0), np.minimum(up, down)).astype(np.float32)


def povey_window(n=400):
    i = np.arange(n, dtype=np.float64)
    hann = 0.5 - 0.5 * np.cos(2 * np.pi * i / (n - 1))
    return (hann ** 0.85).astype(np.float32)


def num_frames(n_samples, win=400, shift=160):
    return 0 if n_samples < win else 1 + (n_samples - win) // shift


def fbank(wave, num_bins=80, sample_freq=16000.0):
    """wave: 1-D float array already scaled to int16 range (×2^15). Returns [T, num_bins] fp32."""
    wave = np.asarray(wave, dtype=np.float32)
    win, shift, padded = 400, 160, 512
    T = num_frames(len(wave), win, shift)
    if T == 0:
        return np.zeros((0, num_bins), np.float32)
    idx = np.arange(T)[:, None] * shift + np.arange(win)[None, :]
    fr = wave[idx].astype(np.float32)
    fr = fr - fr.mean(axis=1, keepdims=True, dtype=np.float32)
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    fr = fr - np.float32(0.97) * prev
    fr = fr * povey_window(win)[None, :]
    fr = np.pad(fr, ((0, 0), (0, padded - win)))
    spec = np.abs(np.fft.rfft(fr.astype(np.float64), axis=1)) ** 2
    banks = np.pad(mel_banks(num_bins, padded, sample_freq), ((0, 0), (0, 1)))
    mel = spec.astype(np.float32) @ banks.T
    return np.log(np.maximum(mel, FLT_EPS)).astype(np.float32)


def utterance_cmvn(x, norm_means=True, norm_vars=True):
    """fairseq UtteranceCMVN.__call__ (per-utterance mean/var over time)."""
    x = np.asarray(x, dtype=np.float32)
    mean = x.mean(axis=0)
    sq = (x ** 2).sum(axis=0)
    if norm_means:
        x = x - mean
    if norm_vars:
        var = sq / x.shape[0] - mean ** 2
        x = x / np.sqrt(np.maximum(var, 1e-10))
    return x.astype(np.float32)


def specaugment(x, draws, n_freq, n_time, mask_value=None):
    """fairseq ``SpecAugmentTransform.__call__`` (data/audio/feature_transforms/specaugment.py;
    time_warp_W = 0) with its random draws given: draws = [f0, f]*n_freq + [t0, t]*n_time, a zero
    width masking nothing; mask value = ``spectrogram.mean()`` of the undistorted input when
    mask_value is None.  x: [T, F] float32 (one utterance, unpadded)."""
    x = np.asarray(x, dtype=np.float32)
    out = x.copy()
    mv = x.mean() if mask_value is None else mask_value
    for k in range(n_freq):
        f0, f = int(draws[2 * k]), int(draws[2 * k + 1])
        if f != 0:
            out[:, f0:f0 + f] = mv
    for k in range(n_time):
        t0, t = int(draws[2 * (n_freq + k)]), int(draws[2 * (n_freq + k) + 1])
        if t != 0:
            out[t0:t0 + t, :] = mv
    return out


def synth_wave(n_frames, rng, tone_hz=440.0):
    """Synthetic utterance of N = 160*T + 240 samples: 0.1*N(0,1)*2^15 + a 440 Hz tone."""
    n = 160 * n_frames + 240
    t = np.arange(n, dtype=np.float64) / 16000.0
    w = 0.1 * rng.standard_normal(n) + 0.3 * np.sin(2 * np.pi * tone_hz * t)
    return (w * 2 ** 15).astype(np.float32)
