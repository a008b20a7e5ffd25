"""CPU: pin the oracle's fusion restatement to golden vectors produced by the REFERENCE's own
fusion code (oracle/gen_golden.py, shimmed import of mm_s2ut/models/{fuse,mm_s2s_transformer}.py)."""
import numpy as np
import pytest
import torch

import os

from conftest import GOLDEN, golden_files
from oracle import ref_model as R


def load_case(path):
    z = np.load(path)
    P = {k[len("param."):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param.")}
    P = {"encoder." + k: v for k, v in P.items()}
    d = int(z["d"])
    cfg = R.base_config(
        encoder_embed_dim=d, image_feat_dim=int(z["Di"]),
        multimodal_attention_type=str(z["att"]), use_selective_gate=bool(z["gate"]),
        SA_image_dropout=float(z["p_img"]), SA_text_dropout=float(z["p_txt"]),
        SA_attention_dropout=float(z["p_attn"]))
    masks = {"fusion.img": torch.from_numpy(z["img_keep"]),
             "fusion.txt": torch.from_numpy(z["txt_keep"]),
             "fusion.attn": torch.from_numpy(z["attn_keep"])}
    img_mask = torch.from_numpy(z["img_mask"]) if z["img_mask"].size else None
    return z, P, cfg, masks, img_mask


@pytest.mark.parametrize("path", golden_files("fusion_"), ids=lambda p: p.split("/")[-1])
def test_fusion_oracle_matches_reference(path):
    z, P, cfg, masks, img_mask = load_case(path)
    P = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    text = torch.from_numpy(z["text"]).clone().requires_grad_(True)
    img = torch.from_numpy(z["img"])
    text_mask = torch.from_numpy(z["text_mask"])
    res = R.fuse_img_feat(P, text, img, img_mask, text_mask, cfg, masks, dtype=torch.float64)
    np.testing.assert_allclose(res.detach().numpy(), z["res"], rtol=1e-10, atol=1e-10)
    (res * torch.from_numpy(z["gout"])).sum().backward()
    np.testing.assert_allclose(text.grad.numpy(), z["grad_text"], rtol=1e-9, atol=1e-10)
    for k in z.files:
        if k.startswith("grad.") and k != "grad_text":
            name = "encoder." + k[len("grad."):]
            g = P[name].grad
            g = np.zeros_like(z[k]) if g is None else g.numpy()
            np.testing.assert_allclose(g, z[k], rtol=1e-9, atol=1e-10, err_msg=name)


@pytest.mark.parametrize("path", golden_files("external_"), ids=lambda p: p.split("/")[-1])
def test_external_transformer_oracle_matches_reference(path):
    """the oracle's ExternalMultimodalTransformerEncoder restatement vs the
    reference's own fuse.py run (oracle/gen_golden.py _make_external_case), float64, exact."""
    z = np.load(path)
    pre = "encoder.multimodal_transformer.0."
    P = {pre + k[len("param."):]: torch.from_numpy(z[k]).clone().requires_grad_(True)
         for k in z.files if k.startswith("param.")}
    N = int(z["N"])
    feats = [torch.from_numpy(z[f"feat{i}"]).clone().requires_grad_(True) for i in range(N)]
    img_mask = torch.from_numpy(z["img_mask"]) if z["img_mask"].size else None
    cfg = R.base_config(SA_attention_dropout=0.0)
    res = R.external_multimodal_transformer(P, feats, torch.from_numpy(z["img"]), torch.from_numpy(z["text_mask"]),
                                            img_mask, cfg, dtype=torch.float64)
    np.testing.assert_allclose(res.detach().numpy(), z["res"], rtol=1e-9, atol=1e-10)
    (res * torch.from_numpy(z["gout"])).sum().backward()
    for i, f in enumerate(feats):
        np.testing.assert_allclose(f.grad.numpy(), z[f"grad_feat{i}"], rtol=1e-8, atol=1e-10)
    for k in z.files:
        if k.startswith("grad."):
            name = pre + k[len("grad."):]
            g = P[name].grad
            g = np.zeros_like(z[k]) if g is None else g.numpy()
            np.testing.assert_allclose(g, z[k], rtol=1e-8, atol=1e-10, err_msg=name)


def _shipped():
    from oracle import gen_golden as G
    z = np.load(os.path.join(GOLDEN, "shipped_fusion.npz"))
    P, X, probes = G.shipped_inputs(int(z["seed"]))
    for k, v in {**P, **X}.items():     # the regenerated arrays are the ones the reference ran on
        if f"digest.{k}" in z.files:
            assert G.array_digest(v) == str(z[f"digest.{k}"]), k
    return G, z, P, X, probes


@pytest.mark.parametrize("att", ["multimodal_attention", "selective_attention"])
def test_shipped_shape_oracle_matches_reference(att):
    """the oracle's fusion restatement at the shipped shape (d = Di = 768,
    Ti = 577 (+ bias_kv), Te = 125, B = 2, text and image padding, gate on) against the reference's
    own float64 run (tests/golden/shipped_fusion.npz); weight gradients through their stored
    sketches G @ R, L^T @ G."""
    G, z, P, X, probes = _shipped()
    tag = "mma" if att == "multimodal_attention" else "sa"
    cfg = R.base_config(multimodal_attention_type=att, use_selective_gate=True, SA_image_dropout=0.0,
                        SA_text_dropout=0.0, SA_attention_dropout=0.0)
    Pm = {k: torch.from_numpy(np.array(v)).clone().requires_grad_(True) for k, v in G.shipped_model_params(P, att).items()}
    text = torch.from_numpy(X["text"]).clone().requires_grad_(True)
    res = R.fuse_img_feat(Pm, text, torch.from_numpy(X["img"]), torch.from_numpy(X["img_mask"]),
                          torch.from_numpy(X["text_mask"]), cfg, {}, dtype=torch.float64)
    np.testing.assert_allclose(res.detach().numpy(), z[f"{tag}.res"], rtol=1e-5, atol=1e-6)
    (res * torch.from_numpy(X["gout"])).sum().backward()
    np.testing.assert_allclose(text.grad.numpy(), z[f"{tag}.grad_text"], rtol=1e-5, atol=1e-6)
    for k in z.files:
        if k.startswith(f"{tag}.grad."):
            g = Pm["encoder." + k[len(tag) + 6:]].grad.numpy().reshape(z[k].shape)
            np.testing.assert_allclose(g, z[k], rtol=1e-5, atol=1e-6, err_msg=k)
        elif k.startswith(f"{tag}.gsk."):
            n = k[len(tag) + 5:]
            g = Pm["encoder." + n].grad.numpy()
            key = n.split(".", 2)[-1] if "attns" in n else n
            R_, L_ = probes[key]
            np.testing.assert_allclose(g @ R_, z[k], rtol=1e-5, atol=1e-5, err_msg=k)
            np.testing.assert_allclose(L_.T @ g, z[f"{tag}.gskT.{n}"], rtol=1e-5, atol=1e-5, err_msg=k)


def qformer_case(path):
    """A reference-run QFormerModel case (oracle/gen_golden.py _make_qformer_case): the oracle
    config, the parameters under the model's names (encoder.q_former.*), inputs time-major."""
    z = np.load(path)
    D = int(z["D"])
    cfg = R.base_config(encoder_embed_dim=D, image_feat_dim=D, multimodal_extractor_type="q_former",
                        num_queries=int(z["Q"]), num_query_layers=int(z["nq"]), num_multimodal_layers=int(z["nm"]),
                        self_attention_first=bool(z["sa_first"]), SA_attention_dropout=0.0)
    P = {R.QF + "." + k[len("param."):]: torch.from_numpy(z[k].astype(np.float64))
         for k in z.files if k.startswith("param.")}
    return z, cfg, P


@pytest.mark.parametrize("path", golden_files("qformer_"), ids=lambda p: p.split("/")[-1])
def test_qformer_oracle_matches_reference(path):
    """the oracle's QFormerModel restatement (oracle/ref_model.py
    qformer, both self_attention_first branches of fuse.py:254-259) vs the reference's own fuse.py
    run in float64 on fp16-representable inputs; results stored as float32, hence rtol 1e-5."""
    z, cfg, P = qformer_case(path)
    P = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    m1 = torch.from_numpy(z["m1"].astype(np.float64)).transpose(0, 1).requires_grad_(True)
    m2 = torch.from_numpy(z["m2"].astype(np.float64)).transpose(0, 1).requires_grad_(True)
    res = R.qformer(P, m1, m2, torch.from_numpy(z["text_mask"]), cfg, dtype=torch.float64).transpose(0, 1)
    np.testing.assert_allclose(res.detach().numpy(), z["res"], rtol=1e-5, atol=1e-6)
    (res * torch.from_numpy(z["gout"].astype(np.float64))).sum().backward()
    np.testing.assert_allclose(m1.grad.transpose(0, 1).numpy(), z["grad_m1"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(m2.grad.transpose(0, 1).numpy(), z["grad_m2"], rtol=1e-5, atol=1e-6)
    for k in z.files:
        if k.startswith("grad.") and k != "grad_m1":
            name = R.QF + "." + k[len("grad."):]
            np.testing.assert_allclose(P[name].grad.numpy(), z[k], rtol=1e-5, atol=1e-6, err_msg=name)
