"""Shared helpers for the model-level GPU parity tests (test infrastructure).

``run_model_pair`` runs one training forward + hand-written backward of the HIP model and the same
step of the CPU oracle (oracle/ref_model.py) on identical fp16-rounded parameters and inputs.
Dropout stays ON: every site's keep-mask is regenerated from the HIP counter RNG (the (seed,
offset) pairs the forward recorded in its contexts) and injected into the oracle, so the two
paths drop exactly the same elements.  The backward runs on a loss-scaled gradient (as the
FP16 trainer always does) and is unscaled before comparison.
"""
import numpy as np
import torch

from oracle import ref_model as R


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def round16(P):
    return {k: v.half().float() for k, v in P.items()}


class _Draws:
    """Forced modality-dropout draws (replaces the model's numpy stream)."""

    def __init__(self, vals):
        self.vals = list(vals)

    def random(self):
        return self.vals.pop(0)


MODALITY_DRAWS = {None: (0.99, 0.99), "audio": (0.0, 0.0), "image": (0.0, 0.99)}


def hip_masks(mm, cfg, ectx, dctx, B, Te, Tt, relu=True):
    """{oracle site: bool keep-mask in the oracle's layout} from the HIP forward contexts; with
    relu=True also each FFN's ReLU activity pattern (``{layer}.relu``, from the stored fp16 fc1
    output, see oracle/ref_model.py _relu)."""
    K = mm.kernels
    d, H, F = cfg["encoder_embed_dim"], cfg["encoder_attention_heads"], cfg["encoder_ffn_embed_dim"]
    dd, Hd, Fd = cfg["decoder_embed_dim"], cfg["decoder_attention_heads"], cfg["decoder_ffn_embed_dim"]
    out = {}

    def m(drop, n, p):
        return K.dropout_mask(n, p, drop[0], drop[1], "cuda").bool().cpu()

    def tb(x, T, C):    # [B*T*C] batch-major -> oracle [T, B, C]
        return x.view(B, T, C).transpose(0, 1)

    pd, pa, pact = cfg["dropout"], cfg["attention_dropout"], cfg["activation_dropout"]
    if pd > 0:
        out["encoder.embed"] = tb(m(ectx["drop_emb"], B * Te * d, pd), Te, d)
    for l, c in enumerate(ectx["layers"]):
        p = f"encoder.transformer_layers.{l}"
        if pa > 0:
            out[p + ".attn"] = m(c["drop_attn"], B * H * Te * Te, pa).view(B * H, Te, Te)
        if pd > 0:
            out[p + ".drop1"] = tb(m(c["drop1"], B * Te * d, pd), Te, d)
            out[p + ".drop2"] = tb(m(c["drop2"], B * Te * d, pd), Te, d)
        if pact > 0:
            out[p + ".act"] = tb(m(c["drop_act"], B * Te * F, pact), Te, F)
        if relu:
            out[p + ".relu"] = tb((c["f1"] > 0).cpu(), Te, F)
    xc = ectx.get("ext")
    if xc is not None:       # external multimodal transformer (oracle external_multimodal_transformer sites)
        Hx = cfg["image_feat_dim"] // 64
        for i, c in enumerate(xc["layers"]):
            p = f"encoder.multimodal_transformer.0.layers.{i}"
            pp, Ti, Fx = c["pp"], c["Ti"], 4 * cfg["image_feat_dim"]
            if pp > 0:
                out[p + ".self_attn"] = m(c["drop_sa"], B * Hx * Te * Te, pp).view(B * Hx, Te, Te)
                out[p + ".cross_attn"] = m(c["drop_ca"], B * Hx * Te * Ti, pp).view(B * Hx, Te, Ti)
                for s_ in ("drop1", "drop2", "drop3"):
                    out[f"{p}.{s_}"] = tb(m(c[s_], B * Te * d, pp), Te, d)
                out[p + ".act"] = tb(m(c["drop_act"], B * Te * Fx, pp), Te, Fx)
    qc = ectx.get("qformer")
    if qc is not None:       # QFormer extractor (oracle qformer / multimodal_decoder_layer sites)
        D = cfg["image_feat_dim"]
        Hq, Q = max(1, D // 64), qc["Q"]
        for grp, lst in (("query_transformer_layers", qc["q"]), ("multimodal_transformer_layers", qc["m"])):
            for i, c in enumerate(lst):
                p, pp, Tm = f"encoder.q_former.{grp}.{i}", c["pp"], c["Ti"]
                if pp > 0:
                    out[p + ".self_attn"] = m(c["drop_sa"], B * Hq * Q * Q, pp).view(B * Hq, Q, Q)
                    out[p + ".cross_attn"] = m(c["drop_ca"], B * Hq * Q * Tm, pp).view(B * Hq, Q, Tm)
                    for s_ in ("drop1", "drop2", "drop3"):
                        out[f"{p}.{s_}"] = tb(m(c[s_], B * Q * D, pp), Q, D)
                    out[p + ".act"] = tb(m(c["drop_act"], B * Q * 4 * D, pp), Q, 4 * D)
    fc = ectx.get("fusion")
    if fc is not None:
        Ti, Di, Tk = fc["Ti"], fc["Di"], fc["Tk"]
        if fc["pimg"] > 0:
            out["fusion.img"] = tb(m(fc["drop_img"], B * Ti * Di, fc["pimg"]), Ti, Di)
        if fc["ptxt"] > 0:
            out["fusion.txt"] = tb(m(fc["drop_txt"], B * Te * d, fc["ptxt"]), Te, d)
        if fc["pat"] > 0:
            out["fusion.attn"] = m(fc["drop_attn"], B * Te * Tk, fc["pat"]).view(B, Te, Tk)
    if pd > 0:
        out["decoder.embed"] = m(dctx["drop_emb"], B * Tt * dd, pd).view(B, Tt, dd)
    for l, c in enumerate(dctx["layers"]):
        p = f"decoder.layers.{l}"
        if pa > 0:
            out[p + ".self_attn"] = m(c["drop_sa"], B * Hd * Tt * Tt, pa).view(B * Hd, Tt, Tt)
            out[p + ".cross_attn"] = m(c["drop_ca"], B * Hd * Tt * Te, pa).view(B * Hd, Tt, Te)
        if pd > 0:
            for s in ("drop1", "drop2", "drop3"):
                out[f"{p}.{s}"] = tb(m(c[s], B * Tt * dd, pd), Tt, dd)
        if pact > 0:
            out[p + ".act"] = tb(m(c["drop_act"], B * Tt * Fd, pact), Tt, Fd)
        if relu:
            out[p + ".relu"] = tb((c["f1"] > 0).cpu(), Tt, Fd)
    return out


class PairResult:
    pass


def run_model_pair(mm, cfg, lengths, tlens, *, img_tokens=37, img_mask=False, with_images=True,
                   seed=0, modality=None, scale="dynamic", taps=True, dropout_seed=1234, replay_relu=True):
    """One step of both paths.  cfg: oracle-style config (R.base_config / R.tiny_config).
    scale: the loss scale of the HIP backward, or "dynamic": fairseq's DynamicLossScaler
    behaviour from its initial 128 — halve and rerun (same dropout seed, same masks) while any
    fp16 gradient overflows."""
    P = round16(R.init_params(cfg, seed=seed + 5, include_unused=False))
    model = mm.MMS2UTModel(mm.default_cfg(**cfg), device="cuda")
    model.params.load_state_dict(P, strict=True)
    sample = mm.data.make_sample(lengths, tlens, img_tokens=img_tokens, img_dim=cfg["image_feat_dim"],
                                 with_images=with_images, img_mask=img_mask, seed=seed)
    ni = sample["net_input"]
    ni["src_tokens"] = ni["src_tokens"].half().float()
    if ni["imgs_list"]:
        ni["imgs_list"][0] = ni["imgs_list"][0].half().float()
    batch = mm.runtime.prepare_batch(sample, model.cfg)
    stash = {"enc_dx": {}, "dec_dx": {}}
    ef, df = model.encoder_forward, model.decoder_forward
    eb, db = model.enc_layer_bwd, model.dec_layer_bwd

    def enc_fwd(b):
        out = ef(b)
        stash["e"] = out[3]
        return out

    def dec_fwd(b, enc, l32, Te):
        out = df(b, enc, l32, Te)
        stash["d"] = out[1]
        return out

    def enc_bwd(l, *a, **k):
        out = eb(l, *a, **k)
        stash["enc_dx"][l] = out[0].float().cpu()
        return out

    def dec_bwd(l, *a, **k):
        out = db(l, *a, **k)
        stash["dec_dx"][l] = out[0].float().cpu()
        return out

    model.encoder_forward, model.decoder_forward = enc_fwd, dec_fwd
    model.enc_layer_bwd, model.dec_layer_bwd = enc_bwd, dec_bwd
    V = cfg["vocab_size"]
    B, Tt = ni["prev_output_tokens"].shape
    s = 128.0 if scale == "dynamic" else float(scale)
    while True:
        model.drop.reset(dropout_seed)
        model.np_rng = _Draws(MODALITY_DRAWS[modality])
        model.params.grad.zero_()
        logits = mm.runtime.model_logits(model, batch)
        Te = batch.Te
        masks = hip_masks(mm, model.cfg, stash["e"], stash["d"], B, Te, Tt, relu=replay_relu)
        loss, nll = mm.runtime.label_smoothed_ce(logits, batch.target, V, cfg["label_smoothing"], 1)
        lg = logits[:, :V].float().cpu().view(B, Tt, V)
        loss.backward(torch.tensor(s, device="cuda"))
        torch.cuda.synchronize()
        if scale != "dynamic" or bool(torch.isfinite(model.params.grad).all()) or s <= 1.0 / 64:
            break
        s /= 2
    r = PairResult()
    r.model, r.sample, r.scale, r.B, r.Te, r.Tt = model, sample, s, B, Te, Tt
    r.lg, r.loss, r.nll = lg, loss.item(), nll.item()
    r.grads = {k: model.params.g[k].float().cpu() / s for k in P}
    r.enc_dx = {l: v / s for l, v in stash["enc_dx"].items()}
    r.dec_dx = {l: v / s for l, v in stash["dec_dx"].items()}
    Pg = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    tp = {} if taps else None
    R.RELU_STATS = [] if replay_relu else None
    try:
        lo, nllo, lgo = R.model_forward(Pg, sample, cfg, masks=masks, modality=modality, taps=tp)
    finally:
        r.relu_stats, R.RELU_STATS = R.RELU_STATS, None
    lo.backward()
    r.lgo, r.lo, r.nllo = lgo.detach(), lo.item(), nllo.item()
    r.ref_grads = {k: v.grad for k, v in Pg.items()}
    r.taps = tp
    r.n_masks = len([k for k in masks if not k.endswith(".relu")])
    return r


def grad_errors(r):
    """{param: relative L2 error} (k_proj biases, mathematically zero, reported vs the v bias)."""
    errs = {}
    for k, ref in r.ref_grads.items():
        g = r.grads[k]
        if ref is None or ref.norm() == 0:
            errs[k] = float(g.norm())      # must be exactly 0
            continue
        if k.endswith("k_proj.bias"):
            vb = r.ref_grads[k.replace("k_proj", "v_proj")]
            errs[k] = float(g.norm() / (vb.norm() + 1e-30))
            continue
        errs[k] = rel(g, ref)
    return errs


def layer_dgrad_errors(r):
    """{"enc{l}" / "dec{l}": relative error of the gradient w.r.t. that layer's input}."""
    out = {}
    B, Te, Tt = r.B, r.Te, r.Tt
    for l, dx in r.enc_dx.items():
        t = r.taps.get(f"enc{l}")
        if t is not None and t.grad is not None:
            out[f"enc{l}"] = rel(dx.view(B, Te, -1), t.grad.transpose(0, 1))
    for l, dx in r.dec_dx.items():
        t = r.taps.get(f"dec{l}")
        if t is not None and t.grad is not None:
            out[f"dec{l}"] = rel(dx.view(B, Tt, -1), t.grad.transpose(0, 1))
    return out


def check_outputs(r, logit_tol=1e-2, loss_tol=2e-3, min_coverage=0.9):
    """Logits / loss tolerances and the unit-token argmax check.  The argmax is compared wherever
    the oracle's top-2 margin exceeds 0.05 (the fp16 noise floor); the check must cover at least
    ``min_coverage`` of the non-pad positions so it cannot pass vacuously —
    the counts land in r.argmax_compared / r.argmax_positions and in report()."""
    assert rel(r.lg, r.lgo) < logit_tol, rel(r.lg, r.lgo)
    keep = r.sample["target"] != 1
    top2 = r.lgo.topk(2, -1).values
    confident = keep & ((top2[..., 0] - top2[..., 1]) > 0.05)
    r.argmax_compared, r.argmax_positions = int(confident.sum()), int(keep.sum())
    assert r.argmax_compared >= min_coverage * r.argmax_positions, (r.argmax_compared, r.argmax_positions)
    assert torch.equal(r.lg.argmax(-1)[confident], r.lgo.argmax(-1)[confident])
    assert abs(r.loss - r.lo) / abs(r.lo) < loss_tol, (r.loss, r.lo)
    assert abs(r.nll - r.nllo) / abs(r.nllo) < loss_tol, (r.nll, r.nllo)


def check_relu_replay(r, max_frac=1e-3):
    """the replayed FFN activity pattern (HIP fc1 output > 0) may depart from
    the fp32 oracle's own pre-activation signs only by rounding flips — in total fewer than
    ``max_frac`` of the compared units, and each flipped unit's |pre-activation| under 5 % of the
    layer's mean |pre-activation| — so the replay cannot hide an fc1 epilogue bug."""
    st = r.relu_stats
    assert st, "no ReLU replay statistics recorded"
    dis, tot = sum(s[1] for s in st), sum(s[2] for s in st)
    r.relu_disagree = (dis, tot)
    assert dis < max_frac * tot, (dis, tot)
    for site, n, t, xmax, xmean in st:
        assert xmax <= 0.05 * xmean, (site, n, t, xmax, xmean)


def report(r, top=12):
    errs = grad_errors(r)
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:top]
    lines = [f"logits rel {rel(r.lg, r.lgo):.2e} loss {r.loss:.6g} vs {r.lo:.6g} masks {r.n_masks} "
             f"loss scale {r.scale:g}"]
    if getattr(r, "argmax_positions", None):
        lines.append(f"  argmax compared at {r.argmax_compared} / {r.argmax_positions} non-pad positions")
    if getattr(r, "relu_stats", None):
        dis, tot = sum(s[1] for s in r.relu_stats), sum(s[2] for s in r.relu_stats)
        flip = max((s[3] / max(s[4], 1e-30) for s in r.relu_stats), default=0.0)
        lines.append(f"  ReLU replay: {dis} sign flips / {tot} units ({dis / max(tot, 1):.2e}); "
                     f"largest flipped |pre-act| / mean |pre-act| = {flip:.2e}")
    lines += [f"  grad {k}: {e:.3e}" for k, e in worst]
    if r.taps:
        lines += [f"  dgrad {k}: {e:.3e}" for k, e in sorted(layer_dgrad_errors(r).items())]
    return "\n".join(lines)


__all__ = ["rel", "round16", "run_model_pair", "grad_errors", "layer_dgrad_errors", "check_outputs",
           "report", "np"]
