"""GPU parity of the multitask auxiliary heads (--multitask-config-yaml,
fairseq MultitaskCriterion as mm_s2ut/criterions/speech_to_speech_criterion.py:94-100 drives it):
a transformer head on encoder_states[0], a CTC head on encoder_states[1] and a CTC head on the
unit decoder's inner_states[1], trained jointly with the main loss.  The HIP path (aux heads in
the flat parameter buffer, csrc/ctc.hip, gradients injected into the hand-written backward) vs
oracle/ref_model.multitask_losses (fp32; torch's F.ctc_loss is the CTC reference).
Tolerances as test_gpu_model.py: losses 2e-3 relative, every parameter gradient 1e-2 relative
L2 with the FFN ReLU patterns replayed (main and auxiliary decoders)."""
import pytest
import torch

from conftest import pkg
from oracle import ref_model as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _tasks(mm, cfg):
    MT = mm.multitask
    letters = MT.Dictionary([chr(ord("a") + i) for i in range(26)] + ["|"])
    raws = {
        "source_letter": {"decoder_type": "transformer", "encoder_layer": 1, "loss_weight": 8.0,
                          "decoder_args": {"decoder_layers": 2, "decoder_embed_dim": 256, "decoder_ffn_embed_dim": 512,
                                           "decoder_attention_heads": 4, "dropout": 0.0}},
        "target_letter_ctc": {"decoder_type": "ctc", "encoder_layer": 2, "loss_weight": 2.0},
        "decoder_target_ctc": {"decoder_type": "ctc", "decoder_layer": 2, "loss_weight": 1.6},
    }
    return letters, [MT.task_model_cfg(n, r, letters, cfg) for n, r in raws.items()]


def _mt_sample(mm, tasks, letters, sample, seed):
    MT = mm.multitask
    g = torch.Generator().manual_seed(seed)
    pos = torch.argsort(sample["id"])              # pos[i]: collated position of original item i
    B = sample["id"].shape[0]
    per = {}
    te = [int(x) for x in mm.runtime.subsampled_lengths(sample["net_input"]["src_lengths"].numpy(), 2)]
    tt = sample["target_lengths"].tolist()
    for t in tasks:
        items = []
        for i in range(B):           # original item i sits at collated position pos[i]
            j = int(pos[i])
            cap = te[j] if t["input_from"] == "encoder" else tt[j]
            n = max(1, min(int(torch.randint(3, 18, (1,), generator=g)), cap // 2))
            ids = torch.randint(4, len(letters), (n,), generator=g)
            if t["type"] != "ctc":
                ids = torch.cat([ids, torch.tensor([letters.eos])])
            items.append(ids)
        per[t["name"]] = (type("D", (), {"collater": staticmethod(lambda s: MT.collate_text_targets(s, letters.pad))}), items)
    return MT.sample_multitask(per, sample["id"])


def test_multitask_heads_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    ocfg = R.no_dropout(R.tiny_config(conv_channels=256))
    cfg = mm.default_cfg(**ocfg)
    letters, tasks = _tasks(mm, cfg)
    cfg["multitask"] = tasks
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=9)
    P = {k: v.float().cpu() for k, v in model.params.state_dict().items() if k in model.params.offsets}
    sample = mm.data.make_sample([160, 131, 97], [41, 30, 22], img_tokens=37, img_dim=768, seed=2)
    sample["multitask"] = _mt_sample(mm, tasks, letters, sample, seed=3)
    ni = sample["net_input"]
    ni["src_tokens"] = ni["src_tokens"].half().float()
    ni["imgs_list"][0] = ni["imgs_list"][0].half().float()
    batch = mm.runtime.prepare_batch(sample, cfg, "cuda")
    stash = {}
    ef, df = model.encoder_forward, model.decoder_forward
    model.encoder_forward = lambda b: stash.setdefault("e", ef(b))

    def dec(b, enc, l32, Te, spec=None):
        out = df(b, enc, l32, Te, spec=spec)
        stash.setdefault("dec", []).append(out)
        return out
    model.decoder_forward = dec
    model.params.grad.zero_()
    logits, aux = mm.runtime.model_outputs(model, batch)
    relu = {}
    B = ni["prev_output_tokens"].shape[0]
    for pre, ctx, T in (("encoder.transformer_layers", stash["e"][3], stash["e"][2]),):
        for l, c in enumerate(ctx["layers"]):
            relu[f"{pre}.{l}.relu"] = (c["f1"] > 0).cpu().view(B, T, -1).transpose(0, 1)
    for logits_, dctx in stash["dec"]:
        sp = dctx["spec"]
        for l, c in enumerate(dctx["layers"]):
            relu[f"{sp.prefix}.layers.{l}.relu"] = (c["f1"] > 0).cpu().view(B, dctx["Tt"], -1).transpose(0, 1)
    alog = {k: v.item() for k, v in model.last_aux_losses.items()}
    loss, nll = mm.runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"], cfg["label_smoothing"], 1)
    scale = 64.0
    (loss + aux).backward(torch.tensor(scale, device="cuda"))
    torch.cuda.synchronize()
    # oracle
    Pg = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    enc, pad, states = R.encoder_forward(Pg, ni["src_tokens"], ni["src_lengths"], ocfg, ni["imgs_list"][0],
                                         masks=relu, return_all_hiddens=True)
    enc_pad = pad if pad.any() else None
    inner = []
    lo_logits = R.decoder_forward(Pg, ni["prev_output_tokens"], enc, enc_pad, ocfg, masks=relu, inner=inner)
    lo, nllo = R.label_smoothed_nll_loss(lo_logits, sample["target"], ocfg["label_smoothing"], 1)
    mt = dict(sample["multitask"], __target_lengths__=sample["target_lengths"])
    ol = R.multitask_losses(Pg, tasks, states, enc_pad, inner, mt, ocfg, masks=relu)
    total = lo + sum(t["weight"] * ol[t["name"]] for t in tasks)
    total.backward()
    assert abs(loss.item() - lo.item()) / lo.item() < 2e-3
    for t in tasks:
        assert abs(alog[t["name"]] - ol[t["name"]].item()) / ol[t["name"]].item() < 2e-3, (t["name"], alog, ol)
    bad = []
    for k, v in Pg.items():
        g = model.params.g[k].float().cpu() / scale
        if v.grad is None or v.grad.norm() == 0:
            if g.norm() > 0:
                bad.append((k, "nonzero"))
            continue
        if k.endswith("k_proj.bias"):
            continue        # mathematically zero (shift-invariant softmax)
        e = _rel(g, v.grad)
        if e > 1e-2:
            bad.append((k, e))
    assert not bad, bad[:10]
    for t in tasks:             # every head received gradient
        name = next(k for k in P if k.startswith(t["name"] + "_decoder"))
        assert model.params.g[name].float().norm() > 0


def test_ctc_kernel_vs_torch():
    """csrc/ctc.hip vs torch F.ctc_loss (fp64, CPU): loss, gradient, an impossible alignment
    (zero_infinity) and repeated labels."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K = mm.kernels
    g = torch.Generator().manual_seed(0)
    B, T, V = 4, 37, 29
    ld = 32
    logits = (2 * torch.randn(B * T, ld, generator=g)).half()
    in_len = torch.tensor([37, 30, 11, 25], dtype=torch.int32)
    tl = torch.tensor([9, 12, 8, 5], dtype=torch.int32)        # utterance 2: 8 labels in 11 frames w/ repeats
    tg = torch.randint(1, V, (B, 12), generator=g)
    tg[2, :8] = torch.tensor([3, 3, 3, 3, 5, 5, 5, 5])         # needs 15 frames > 11: impossible
    tg[0, 3] = tg[0, 2]                                         # a repeat that fits
    loss = torch.zeros(1, device="cuda")
    lg = logits.cuda()
    work = K.ctc_loss_fwd(lg, B, T, V, tg.cuda(), in_len.cuda(), tl.cuda(), 12, 0, True, loss)
    gs = torch.tensor([3.0], device="cuda")
    d = K.ctc_loss_bwd(lg, B, T, V, tg.cuda(), in_len.cuda(), tl.cuda(), 12, 0, work, gs)
    torch.cuda.synchronize()
    x = logits[:, :V].double().view(B, T, V).transpose(0, 1).clone().requires_grad_(True)
    lp = torch.log_softmax(x, -1)
    flat = torch.cat([tg[b, :tl[b]] for b in range(B)])
    ref = torch.nn.functional.ctc_loss(lp, flat, in_len.long(), tl.long(), blank=0, reduction="sum", zero_infinity=True)
    (3.0 * ref).backward()
    assert abs(loss.item() - ref.item()) / ref.item() < 1e-4
    dg = d.float().cpu().view(B, T, ld)
    assert _rel(dg[..., :V], x.grad.transpose(0, 1)) < 2e-3
    assert dg[..., V:].abs().max() == 0 and dg[2].abs().max() == 0      # padding columns, impossible row
    assert dg[1, 30:].abs().max() == 0                                  # frames past the input length


def test_ctc_kernel_large_vocab_deterministic():
    """the CTC gradient no longer keeps per-vocabulary LDS tables (a subword target
    dictionary of 10k+ entries used to fail), and loss / gradient are bit-reproducible (no float
    atomics): V = 12000, two runs bit-identical, both equal to torch fp64."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    K = pkg("kernels")
    g = torch.Generator().manual_seed(3)
    B, T, V, S = 3, 60, 12000, 20
    ld = 12000
    logits = (2 * torch.randn(B * T, ld, generator=g)).half()
    in_len = torch.tensor([60, 51, 44], dtype=torch.int32)
    tl = torch.tensor([20, 13, 17], dtype=torch.int32)
    tg = torch.randint(1, V, (B, S), generator=g)
    tg[1, 4:8] = 777                                            # repeated label
    lg, tgd, il, tld = logits.cuda(), tg.cuda(), in_len.cuda(), tl.cuda()
    outs = []
    for _ in range(2):
        loss = torch.zeros(1, device="cuda")
        work = K.ctc_loss_fwd(lg, B, T, V, tgd, il, tld, S, 0, True, loss)
        d = K.ctc_loss_bwd(lg, B, T, V, tgd, il, tld, S, 0, work, torch.tensor([1.0], device="cuda"))
        torch.cuda.synchronize()
        outs.append((loss.cpu(), d.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    x = logits.double().view(B, T, V).transpose(0, 1).clone().requires_grad_(True)
    flat = torch.cat([tg[b, :tl[b]] for b in range(B)])
    ref = torch.nn.functional.ctc_loss(torch.log_softmax(x, -1), flat, in_len.long(), tl.long(), blank=0,
                                       reduction="sum", zero_infinity=True)
    ref.backward()
    assert abs(outs[0][0].item() - ref.item()) / ref.item() < 1e-4
    assert _rel(outs[0][1].float().view(B, T, ld), x.grad.transpose(0, 1)) < 2e-3
