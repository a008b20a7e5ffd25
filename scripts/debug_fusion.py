"""Stage-by-stage check of the fusion block on the GPU against torch fp32 (debug tool)."""
import importlib, sys, os
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mm = importlib.import_module("multimodal-s2ut_amd")
K = mm.kernels
def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu(); return ((a - b).norm() / (b.norm() + 1e-12)).item()
z = np.load(sys.argv[1])
d, Di = int(z["d"]), int(z["Di"])
cfg = mm.default_cfg(encoder_embed_dim=d, encoder_layers=0, decoder_layers=0, image_feat_dim=Di,
                     multimodal_attention_type=str(z["att"]), use_selective_gate=bool(z["gate"]),
                     SA_image_dropout=0.0, SA_text_dropout=0.0, SA_attention_dropout=0.0,
                     conv_channels=16, decoder_embed_dim=d, vocab_size=8)
model = mm.MMS2UTModel(cfg, device="cuda")
sd = {"encoder." + k[len("param."):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param.")}
model.params.load_state_dict(sd, strict=False)
Te, B, _ = z["text"].shape; Ti = z["img"].shape[0]
text = torch.from_numpy(z["text"]).transpose(0, 1).reshape(B * Te, d).cuda().half().contiguous()
img = torch.from_numpy(z["img"]).transpose(0, 1).cuda().half().contiguous()
res, c = model.fusion_fwd(text, img, None, B, Te)
torch.cuda.synchronize()
f = lambda t: t.float().cpu()
P = {k: f(v) for k, v in sd.items()}
pre = c["pre"]
# reference per stage (fp32 on the fp16 inputs)
imgn = torch.nn.functional.layer_norm(f(img).view(B * Ti, Di), (Di,), P["encoder.image_pre_norm_module.weight"], P["encoder.image_pre_norm_module.bias"], 1e-5)
print("imgd", rel(c["imgd"].view(B, -1, Di)[:, :Ti].reshape(B * Ti, Di), imgn))
if c["extra"]:
    W = P[pre + ".in_proj_weight"] if (pre + ".in_proj_weight") in P else torch.cat([P[pre + ".q_proj_weight"], P[pre + ".k_proj_weight"], P[pre + ".v_proj_weight"]])
    bq = P[pre + ".in_proj_bias"]
    q = f(text) @ W[:d].t() + bq[:d]
    kv = imgn @ W[d:].t() + bq[d:]
else:
    q = f(text) @ P[pre + ".q_proj.weight"].t() + P[pre + ".q_proj.bias"]
    kv = torch.cat([imgn @ P[pre + ".k_proj.weight"].t() + P[pre + ".k_proj.bias"], imgn @ P[pre + ".v_proj.weight"].t() + P[pre + ".v_proj.bias"]], 1)
print("q", rel(c["q"], q))
kvg = c["kv"].view(B, c["Tk"], 2 * d)[:, :Ti].reshape(B * Ti, 2 * d)
print("kv", rel(kvg, kv))
for b in range(B):
    print(" kv batch", b, rel(kvg.view(B, Ti, 2 * d)[b], kv.view(B, Ti, 2 * d)[b]))
Tk = c["Tk"]; ldS = c["ldS"]
qq = f(c["q"]).view(B, Te, d); kk = f(c["kv"]).view(B, Tk, 2 * d)[..., :d]; vv = f(c["kv"]).view(B, Tk, 2 * d)[..., d:]
s = qq @ kk.transpose(1, 2) * d ** -0.5
p = torch.softmax(s, -1)
Pg = f(c["P"]).view(B, Te, ldS)[..., :Tk]
print("P", rel(Pg, p))
for b in range(B):
    print(" P batch", b, rel(Pg[b], p[b]))
o = p @ vv
print("O", rel(c["O"], o.reshape(B * Te, d)))
for b in range(B):
    print(" O batch", b, rel(f(c["O"]).view(B, Te, d)[b], o[b]))
ref = torch.from_numpy(z["res"]).transpose(0, 1).reshape(B * Te, d)
print("res", rel(res, ref))
