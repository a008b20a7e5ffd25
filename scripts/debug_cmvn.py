import importlib, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
from oracle import ref_fbank as RF
fe = mm.frontend.FbankFrontend("cuda")
rng = np.random.default_rng(4)
frames = [80, 120, 31]
waves = [RF.synth_wave(T, rng) for T in frames]
wb = fe.upload(waves)
out = fe(wb).float().cpu().numpy()
raw = fe.features_f32(wb).cpu().numpy()
off = wb["frame_off"].cpu().numpy()
for j, i in enumerate(wb["order"]):
    r = RF.fbank(waves[i]); ref = RF.utterance_cmvn(r)
    T = ref.shape[0]
    d = np.abs(out[j, :T] - ref)
    t, c = np.unravel_index(d.argmax(), d.shape)
    print(j, i, T, "max", d.max(), "at", t, c, out[j, t, c], ref[t, c], "raw", raw[off[j] + t, c], r[t, c])
    print("  col stats gpu-raw mean/std", raw[off[j]:off[j+1], c].mean(), raw[off[j]:off[j+1], c].std(), " ref", r[:, c].mean(), r[:, c].std())
