"""GPU: the on-disk data path end to end.  WAV files -> prefetching loader ->
pinned upload -> HIP fbank + CMVN (+ SpecAugment) -> fp16 src_tokens, checked per utterance against
oracle/ref_fbank.py (fbank, utterance_cmvn, specaugment restatements) with the same tolerances as
tests/test_gpu_frontend.py; targets and image rows against the files; then training steps on the
loader's batches.  SpecAugment: unmasked values bit-identical, masked values = the utterance mean
(|err| <= 2e-3, fp16 of an fp32 mean whose summation order differs from numpy's), padding untouched."""
import numpy as np
import pytest
import torch

from conftest import pkg
from manifest_corpus import write_corpus
from oracle import ref_fbank as RF
from oracle import ref_model as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _cmvn_close(got, wave):
    raw = RF.fbank(wave)
    ref = RF.utterance_cmvn(raw)
    cond = raw.mean(0).astype(np.float64) ** 2 / np.maximum(raw.var(0, dtype=np.float64), 1e-10)
    tol = 5e-3 + 2e-7 * cond[None, :] * np.sqrt(ref.shape[0]) * (np.abs(ref) + 1.0)
    err = np.abs(got - ref)
    assert np.all(err <= tol), float(err.max())


def test_loader_matches_oracle(tmp_path):
    mm = pkg()
    M = mm.manifest
    c = write_corpus(str(tmp_path), frames=(120, 57, 200, 57, 88, 31), di=768, ti=17)
    ds = M.MultiModalS2SManifest(str(tmp_path), "train", M.UnitDictionary.for_codes(1000),
                                 image_feat_path=c["feat_dir"])
    cfg = mm.default_cfg(**R.tiny_config(conv_channels=256))
    batches = ds.batches(max_tokens=450)
    assert len(batches) >= 2
    seen = []
    for batch, sample in M.DeviceLoader(ds, batches, cfg, "cuda:0"):
        src = batch.src.float().cpu().numpy()
        ids = sample["id"].tolist()
        assert src.shape[0] == len(ids) and src.shape[1] == max(c["frames"][i] for i in ids)
        for j, i in enumerate(ids):
            T = c["frames"][i]
            _cmvn_close(src[j, :T], c["waves"][i])
            assert np.all(src[j, T:] == 0)
        assert torch.equal(batch.target.cpu(), sample["target"])
        img = sample["net_input"]["imgs_list"][0]
        assert torch.equal(batch.imgs.cpu(), img.half())
        for j, i in enumerate(ids):
            assert torch.equal(img[j], c["feats"][int(c["rows"][i])])
        seen += ids
    assert sorted(seen) == list(range(6))


def test_specaugment_kernel_matches_oracle():
    mm = pkg()
    K, fe_mod = mm.kernels, mm.frontend
    rng = np.random.default_rng(2)
    frames = [300, 120, 31, 5]
    fe = fe_mod.FbankFrontend("cuda:0")
    wb = fe.upload([RF.synth_wave(T, rng) for T in frames])
    base = fe(wb)
    sa = fe_mod.SpecAugment(freq_mask_N=2, freq_mask_F=27, time_mask_N=2, time_mask_T=100, time_mask_p=1.0)
    draws = sa.draws(wb["n_frames"].tolist(), 80, np.random.RandomState(7))
    draws[0, :2] = (3, 26)            # a mask that starts mid-group of 4 bins
    draws[1, 4:6] = (0, 0)            # a zero-width time mask
    masks = torch.from_numpy(draws).cuda()
    for mv in (None, -0.5):
        x = base.clone()
        K.specaugment(x, wb["frame_off"], masks, 2, 2, mv)
        torch.cuda.synchronize()
        got, before = x.float().cpu().numpy(), base.float().cpu().numpy()
        for b, T in enumerate(wb["n_frames"].tolist()):
            ref = RF.specaugment(before[b, :T], draws[b], 2, 2, mask_value=mv)
            masked = RF.specaugment(np.zeros((T, 80), np.float32), draws[b], 2, 2, mask_value=1.0) != 0
            assert np.array_equal(got[b, :T][~masked], before[b, :T][~masked])
            tol = 0.0 if mv is not None else 2e-3
            assert np.abs(got[b, :T][masked] - ref[masked]).max(initial=0.0) <= tol
            assert np.all(got[b, T:] == 0)


def test_training_on_manifest_batches(tmp_path):
    mm = pkg()
    M = mm.manifest
    sa = {"freq_mask_F": 27, "freq_mask_N": 1, "time_mask_N": 1, "time_mask_T": 100, "time_mask_p": 1.0}
    cfgd = R.tiny_config(conv_channels=256)
    c = write_corpus(str(tmp_path), frames=(150, 97, 200, 61, 88, 131, 45), di=cfgd["image_feat_dim"], ti=17,
                     transforms=("utterance_cmvn", "specaugment"), specaugment=sa)
    ds = M.MultiModalS2SManifest(str(tmp_path), "train", M.UnitDictionary.for_codes(1000),
                                 image_feat_path=c["feat_dir"])
    cfg = mm.default_cfg(**cfgd)
    model = mm.MMS2UTModel(cfg, device="cuda:0").init_params(seed=4)
    tr = mm.trainer.Trainer(model, lr=1e-3, warmup_updates=2, world_size=1)
    losses = []
    for epoch in (1, 2):
        for batch, _ in M.DeviceLoader(ds, ds.batches(max_tokens=500, epoch=epoch), cfg, "cuda:0", epoch=epoch):
            log = tr.train_step(batch)
            losses.append(float(log[0] / log[2]))
    torch.cuda.synchronize()
    assert len(losses) >= 4 and all(np.isfinite(losses))
    assert not tr.opt.stats()["fatal"]
