"""CPU: the on-disk data path's host logic — TSV manifest, unit dictionary,
16-bit WAV reading, image-feature rows, length filtering and batching, config transforms, the
SpecAugment mask draws and the SpecAugment restatement.  The GPU half (fbank/CMVN/SpecAugment on
the device vs oracle/ref_fbank.py) is tests/test_gpu_manifest.py."""
import math
import os

import numpy as np
import pytest
import torch

from conftest import pkg
from manifest_corpus import write_corpus
from oracle import ref_fbank as RF


@pytest.fixture()
def M():
    return pkg("manifest")


def test_tsv_and_dictionary(tmp_path, M):
    c = write_corpus(str(tmp_path))
    s = M.load_samples_from_tsv(str(tmp_path), "train")
    assert [r["id"] for r in s] == [f"utt{k}" for k in range(5)]
    assert [int(r["src_n_frames"]) for r in s] == c["frames"]
    d = M.UnitDictionary.for_codes(1000)
    assert len(d) == 1004 and d.pad() == 1 and d.eos() == 2
    # fairseq Dictionary.encode_line: whitespace-normalised split, unk for unknown symbols, eos appended
    assert d.encode_line("  5 17\t999 x ").tolist() == [9, 21, 1003, 3, 2]
    assert d.encode_line("").tolist() == [2]
    with pytest.raises(FileNotFoundError):
        M.load_samples_from_tsv(str(tmp_path), "valid")
    open(os.path.join(tmp_path, "empty.tsv"), "w").write("id\tsrc_audio\n")
    with pytest.raises(ValueError):
        M.load_samples_from_tsv(str(tmp_path), "empty")


def test_wav_roundtrip_is_exact(tmp_path, M):
    rng = np.random.default_rng(1)
    w = rng.integers(-32768, 32768, 4001).astype(np.float32)
    p = os.path.join(tmp_path, "a.wav")
    M.write_wav(p, w)
    x, sr = M.read_wav(p)
    assert sr == 16000 and x.dtype == np.float32 and np.array_equal(x, w)


def test_items_images_and_collate(tmp_path, M):
    c = write_corpus(str(tmp_path))
    ds = M.MultiModalS2SManifest(str(tmp_path), "train", M.UnitDictionary.for_codes(1000),
                                 image_feat_path=c["feat_dir"])
    assert ds.cmvn and ds.specaugment is None and ds.is_train
    for i in range(len(ds)):
        it = ds.item(i)
        assert np.array_equal(it["wave"], c["waves"][i])
        assert it["n_frames"] == c["frames"][i]
        assert it["target"].tolist() == [int(u) + 4 for u in c["units"][i]] + [2]
        row = int(c["rows"][i])          # the WAV is named {row + 1}.wav
        assert ds.image_row(i) == row
        assert torch.equal(it["img"], c["feats"][row])
        assert torch.equal(it["img_mask"], c["mask"][row])
    sample, waves = ds.collate([0, 1, 2, 3, 4])
    ids = sample["id"].tolist()
    lens = sample["net_input"]["src_lengths"].tolist()
    assert lens == sorted(lens, reverse=True) and sorted(ids) == [0, 1, 2, 3, 4]
    assert sample["net_input"]["src_tokens"] is None       # features come from the GPU front end
    for j, i in enumerate(ids):                              # waves follow the collater's order
        assert np.array_equal(waves[j], c["waves"][i]) and lens[j] == c["frames"][i]
        assert torch.equal(sample["net_input"]["imgs_list"][0][j], c["feats"][int(c["rows"][i])])
        t = sample["target"][j]
        n = int(sample["target_lengths"][j])
        assert t[:n].tolist() == [int(u) + 4 for u in c["units"][i]] + [2] and bool((t[n:] == 1).all())
        assert sample["net_input"]["prev_output_tokens"][j, 0] == 2
    assert sample["ntokens"] == sum(len(u) + 1 for u in c["units"])


def test_ordering_filtering_batching(tmp_path, M):
    c = write_corpus(str(tmp_path), frames=(120, 57, 200, 57, 88, 300, 41))
    d = M.UnitDictionary.for_codes(1000)
    ev = M.MultiModalS2SManifest(str(tmp_path), "train", d, is_train=False)
    o = ev.ordered_indices()
    assert [c["frames"][i] for i in o] == sorted(c["frames"], reverse=True)
    assert o.tolist().index(1) < o.tolist().index(3)              # ties keep manifest order (eval)
    b = ev.batches(max_tokens=400)
    assert sorted(sum(b, [])) == list(range(7))
    for bb in b:
        assert len(bb) * max(c["frames"][i] for i in bb) <= 400
    tr = M.MultiModalS2SManifest(str(tmp_path), "train", d)
    assert [c["frames"][i] for i in tr.ordered_indices(seed=1, epoch=3)] == sorted(c["frames"], reverse=True)
    small = M.MultiModalS2SManifest(str(tmp_path), "train", d, max_source_positions=150)
    with pytest.raises(ValueError):
        small.batches(max_tokens=4000)
    kept = sum(small.batches(max_tokens=4000, skip_invalid=True), [])
    assert sorted(kept) == [i for i, T in enumerate(c["frames"]) if T <= 150]


def test_config_transforms(tmp_path, M):
    d = M.UnitDictionary.for_codes(1000)
    sa = {"freq_mask_F": 27, "freq_mask_N": 1, "time_mask_N": 1, "time_mask_T": 100, "time_mask_p": 1.0}
    write_corpus(str(tmp_path), transforms=("utterance_cmvn", "specaugment"), specaugment=sa)
    tr = M.MultiModalS2SManifest(str(tmp_path), "train", d)
    assert tr.cmvn and tr.specaugment is not None and (tr.specaugment.fn, tr.specaugment.ff) == (1, 27)
    ev = M.MultiModalS2SManifest(str(tmp_path), "train", d, is_train=False)   # '*' list: no specaugment
    assert ev.cmvn and ev.specaugment is None
    write_corpus(str(tmp_path), transforms=("specaugment", "utterance_cmvn"), specaugment=sa)
    with pytest.raises(NotImplementedError):
        M.MultiModalS2SManifest(str(tmp_path), "train", d)
    write_corpus(str(tmp_path), transforms=("global_cmvn",))
    with pytest.raises(NotImplementedError):
        M.MultiModalS2SManifest(str(tmp_path), "train", d)


def test_specaugment_draws_follow_the_transform():
    fe = pkg("frontend")
    sa = fe.SpecAugment.from_config_dict({"freq_mask_F": 27, "freq_mask_N": 2, "time_mask_N": 2,
                                          "time_mask_T": 100, "time_mask_p": 0.2})
    rng = np.random.RandomState(5)
    T = [500, 120, 4, 1]
    m = sa.draws(T, 80, rng)
    assert m.shape == (4, 8) and m.dtype == np.int32
    for b, t in enumerate(T):
        for k in range(2):
            f0, f = m[b, 2 * k: 2 * k + 2]
            assert 0 <= f < 27 and 0 <= f0 and f0 + f <= 80
        max_t = min(100, math.floor(t * 0.2))
        for k in range(2):
            t0, w = m[b, 4 + 2 * k: 6 + 2 * k]
            if max_t < 1:
                assert t0 == 0 and w == 0
            else:
                assert 0 <= w < max_t and t0 + w <= t
    # same draws as the transform's own np.random sequence for one utterance
    rng = np.random.RandomState(11)
    got = sa.draws([300], 80, rng)[0]
    r = np.random.RandomState(11)
    ref = []
    for _ in range(2):
        f = r.randint(0, 27)
        ref += [r.randint(0, 80 - f), f]
    for _ in range(2):
        t = r.randint(0, 60)
        ref += [r.randint(0, 300 - t), t]
    assert got.tolist() == ref
    with pytest.raises(NotImplementedError):
        fe.SpecAugment(time_warp_W=5)


def test_specaugment_oracle_known_answer():
    x = np.arange(12, dtype=np.float32).reshape(4, 3)
    y = RF.specaugment(x, [1, 1, 2, 1], 1, 1)          # column 1, row 2, value = mean 5.5
    ref = x.copy()
    ref[:, 1] = 5.5
    ref[2, :] = 5.5
    assert np.array_equal(y, ref)
    assert np.array_equal(RF.specaugment(x, [0, 0, 1, 0], 1, 1), x)   # zero widths mask nothing
    assert np.array_equal(RF.specaugment(x, [0, 3, 0, 0], 1, 1, mask_value=-1.0), np.full_like(x, -1.0))


def test_wav_stereo_downmix_and_format_errors(tmp_path, M):
    """Multi-channel 16-bit WAV -> channel mean (float32); 8-bit PCM and non-16 kHz rejected loudly."""
    import wave
    rng = np.random.default_rng(2)
    st = rng.integers(-30000, 30000, (500, 2)).astype("<i2")
    p = os.path.join(tmp_path, "st.wav")
    with wave.open(p, "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(st.tobytes())
    x, sr = M.read_wav(p)
    assert sr == 16000 and np.array_equal(x, st.astype(np.float32).mean(axis=1, dtype=np.float32))
    p8 = os.path.join(tmp_path, "u8.wav")
    with wave.open(p8, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(1)
        w.setframerate(16000)
        w.writeframes(bytes(range(200)))
    with pytest.raises(ValueError, match="16-bit"):
        M.read_wav(p8)


def test_non_16k_audio_and_short_utterance_rejected(tmp_path, M):
    c = write_corpus(str(tmp_path), frames=(40, 50))
    ds = M.MultiModalS2SManifest(str(tmp_path), "train", M.UnitDictionary.for_codes(1000))
    wav0 = ds.audio_paths[0]
    M.write_wav(wav0, c["waves"][0], sample_rate=8000)
    with pytest.raises(ValueError, match="16 kHz"):
        ds.item(0)
    M.write_wav(wav0, np.zeros(300, np.float32))      # < 400 samples: no fbank frame
    with pytest.raises(ValueError, match="shorter than one"):
        ds.collate([0, 1])


def test_specaugment_short_utterance_draws_no_time_mask():
    fe = pkg("frontend")
    sa = fe.SpecAugment(freq_mask_N=1, freq_mask_F=5, time_mask_N=2, time_mask_T=100, time_mask_p=0.2)
    m = sa.draws([4, 3], 80, np.random.RandomState(0))     # floor(T * 0.2) < 1: no time masks
    assert (m[:, 2:] == 0).all() and (m[:, 1] < 5).all()
