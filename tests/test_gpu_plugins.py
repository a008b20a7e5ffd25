"""GPU: the plugin surface end to end — task -> model -> criterion built from the canonical command
line (tiny sizes) against the oracle, and the mms2ut-train CLI for a few updates.
Tolerances as tests/test_gpu_model.py (loss relative error < 2e-3)."""
import json

import pytest
import torch

from conftest import pkg
from oracle import ref_model as R
from test_plugins import FUSION_YAML

pytestmark = pytest.mark.gpu

TINY = ("--encoder-layers 2 --decoder-layers 2 --encoder-embed-dim 256 --encoder-ffn-embed-dim 1024 "
        "--encoder-attention-heads 4 --decoder-attention-heads 4")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _args(tmp_path, extra=""):
    y = tmp_path / "mm.yaml"
    y.write_text(FUSION_YAML.replace("SA_image_dropout: 0.1", "SA_image_dropout: 0.0")
                 .replace("SA_attention_dropout: 0.1", "SA_attention_dropout: 0.0"))
    argv = (f"/d --task multimodal_speech_to_speech --arch mm_s2ut_transformer --criterion speech_to_unit "
            f"--target-is-code --target-code-size 1000 --share-decoder-input-output-embed --dropout 0.0 "
            f"--attention-dropout 0.0 --relu-dropout 0.0 --fp16 --multimodal-translation-config-yaml {y} "
            f"{TINY} {extra}")
    return pkg("plugins").build_parser().parse_args(argv.split())


def test_plugin_task_model_criterion_vs_oracle(tmp_path):
    P = pkg("plugins")
    mm = pkg()
    a = _args(tmp_path)
    task = P.REGISTRY["task"][a.task].setup_task(a)
    model = task.build_model(a)
    crit = P.REGISTRY["criterion"]["speech_to_speech"](task, a.label_smoothing)
    cfg = {k: v for k, v in model.cfg.items()}
    ocfg = R.no_dropout(R.tiny_config())
    for k in ocfg:
        assert cfg[k] == ocfg[k] or k in ("max_target_positions",), (k, cfg[k], ocfg[k])
    Pp = {k: v.half().float() for k, v in R.init_params(ocfg, seed=11, include_unused=False).items()}
    model.load_state_dict(Pp, strict=True)
    sample = mm.data.make_sample([300, 211, 160], [91, 64, 49], img_tokens=37, img_dim=768, seed=3)
    ni = sample["net_input"]
    ni["src_tokens"] = ni["src_tokens"].half().float()
    ni["imgs_list"][0] = ni["imgs_list"][0].half().float()
    model.eval()
    logits, extra = model(**ni)
    assert logits.shape == (3, ni["prev_output_tokens"].shape[1], 1004)
    model.train()
    loss, ss, lo = crit(model, sample)
    assert ss == sample["ntokens"] and lo["nsentences"] == 3
    loss.backward()
    torch.cuda.synchronize()
    ref_loss, ref_nll, _ = R.model_forward(Pp, sample, ocfg)
    assert abs(loss.item() - ref_loss.item()) / ref_loss.item() < 2e-3
    assert abs(lo["nll_loss"].item() - ref_nll.item()) / ref_nll.item() < 2e-3
    g = model.net.params.grad.float()
    assert torch.isfinite(g).all() and g.norm() > 0
    # state_dict round trip keeps fairseq names
    sd = model.state_dict()
    for k in ("encoder.transformer_layers.0.self_attn.q_proj.weight", "decoder.embed_tokens.weight",
              "encoder.multimodal_attns.0.bias_k", "encoder.subsample.conv_layers.0.weight"):
        assert k in sd, k
    assert torch.equal(sd["decoder.embed_tokens.weight"].float().cpu(), Pp["decoder.embed_tokens.weight"])


def test_cli_trains_synthetic(tmp_path, capsys):
    a = _args(tmp_path)
    y = a.multimodal_translation_config_yaml
    argv = (f"/d --task multimodal_speech_to_speech --arch mm_s2ut_transformer --criterion speech_to_unit "
            f"--target-is-code --target-code-size 1000 --share-decoder-input-output-embed --fp16 "
            f"--multimodal-translation-config-yaml {y} {TINY} --max-update 6 --max-tokens 6000 "
            f"--log-interval 3 --warmup-updates 4 --lr 1e-3 --synthetic").split()
    assert pkg("cli").main(argv) == 0
    recs = [json.loads(l) for l in capsys.readouterr().out.splitlines() if l.startswith("{")]
    assert [r["num_updates"] for r in recs] == [3, 6]
    for r in recs:
        assert r["loss"] > 0 and r["nll_loss"] > 0 and r["loss_scale"] > 0
        assert r["wps"] > 0


def test_cli_trains_on_manifest(tmp_path, capsys):
    """mms2ut-train DATA ...: TSV + WAVs + config.yaml (utterance_cmvn, specaugment) + .pth image
    features named by the fusion YAML — the on-disk path of SURVEY §8f row 1."""
    from manifest_corpus import write_corpus
    sa = {"freq_mask_F": 27, "freq_mask_N": 1, "time_mask_N": 1, "time_mask_T": 100, "time_mask_p": 1.0}
    d = tmp_path / "data"
    d.mkdir()
    c = write_corpus(str(d), frames=(150, 97, 200, 61, 88, 131, 45, 170), di=768, ti=12,
                     transforms=("utterance_cmvn", "specaugment"), specaugment=sa)
    y = tmp_path / "mm.yaml"
    y.write_text(FUSION_YAML.replace('["/feats/vit_base_patch16_384"]', f'["{c["feat_dir"]}"]'))
    argv = (f"{d} --task multimodal_speech_to_speech --arch mm_s2ut_transformer --criterion speech_to_unit "
            f"--config-yaml config.yaml --target-is-code --target-code-size 1000 "
            f"--share-decoder-input-output-embed --fp16 --multimodal-translation-config-yaml {y} {TINY} "
            f"--max-update 5 --max-tokens 600 --log-interval 5 --warmup-updates 4 --lr 1e-3").split()
    assert pkg("cli").main(argv) == 0
    recs = [json.loads(l) for l in capsys.readouterr().out.splitlines() if l.startswith("{")]
    assert [r["num_updates"] for r in recs] == [5]
    assert recs[0]["loss"] > 0 and recs[0]["wps"] > 0


def _tiny_model(tmp_path, seed=11):
    P = pkg("plugins")
    a = _args(tmp_path)
    task = P.REGISTRY["task"][a.task].setup_task(a)
    model = task.build_model(a)
    ocfg = R.no_dropout(R.tiny_config())
    Pp = {k: v.half().float() for k, v in R.init_params(ocfg, seed=seed, include_unused=False).items()}
    model.load_state_dict(Pp, strict=True)
    return P, model, ocfg, Pp


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_return_all_hiddens_and_encoder_out_contract(tmp_path):
    """mm_s2s_transformer.py:643-665 / :697-699: forward(return_all_hiddens=True) puts the L_e
    per-layer encoder states and the padding mask in extra; forward_encoder returns fairseq's
    encoder-out dict; reorder_encoder_out selects batch entries in every field."""
    P, model, ocfg, Pp = _tiny_model(tmp_path)
    mm = pkg()
    sample = mm.data.make_sample([300, 211, 160], [91, 64, 49], img_tokens=37, img_dim=768, seed=3)
    ni = sample["net_input"]
    ni["src_tokens"] = ni["src_tokens"].half().float()
    ni["imgs_list"][0] = ni["imgs_list"][0].half().float()
    model.train()
    logits, extra = model(**ni, return_all_hiddens=True, target=sample["target"])
    enc_o, pad_o, states_o = R.encoder_forward(Pp, ni["src_tokens"], ni["src_lengths"], ocfg,
                                               imgs=ni["imgs_list"][0], return_all_hiddens=True)
    assert len(extra["encoder_states"]) == ocfg["encoder_layers"] == len(states_o)
    for s, so in zip(extra["encoder_states"], states_o):
        assert s.shape == so.shape and _rel(s, so) < 1e-2
    assert torch.equal(extra["encoder_padding_mask"][0].cpu(), pad_o)
    logits.sum().backward()                 # the states do not break the fused backward
    torch.cuda.synchronize()
    model.eval()
    eo = model.forward_encoder(ni["src_tokens"], ni["src_lengths"], imgs_list=ni["imgs_list"],
                               img_masks_list=ni["img_masks_list"], return_all_hiddens=True)
    assert set(eo) == {"encoder_out", "encoder_padding_mask", "encoder_embedding", "encoder_states",
                       "src_tokens", "src_lengths"}
    assert eo["encoder_out"][0].shape == enc_o.shape and _rel(eo["encoder_out"][0], enc_o) < 1e-2
    assert torch.equal(eo["encoder_padding_mask"][0].cpu(), pad_o)
    order = torch.tensor([2, 0, 0, 1], device="cuda")
    ro = model.reorder_encoder_out(eo, order)
    assert torch.equal(ro["encoder_out"][0], eo["encoder_out"][0].index_select(1, order))
    assert torch.equal(ro["encoder_padding_mask"][0], eo["encoder_padding_mask"][0][order])
    assert len(ro["encoder_states"]) == 2 and ro["encoder_states"][1].shape[1] == 4
    # a batch without padding: fairseq's [] mask
    one = model.forward_encoder(ni["src_tokens"][:1, :300], ni["src_lengths"][:1],
                                imgs_list=[ni["imgs_list"][0][:1]], img_masks_list=[None])
    assert one["encoder_padding_mask"] == [] and one["encoder_states"] == []


def test_decoder_adapter_incremental_matches_full_prefix(tmp_path):
    """fairseq's incremental-decoder protocol through model.decoder: per-step logits with an
    incremental_state (HIP KV-cache decoder) equal the full-prefix decode at the last position,
    across a reorder_incremental_state that permutes and drops hypotheses."""
    P, model, ocfg, Pp = _tiny_model(tmp_path, seed=12)
    mm = pkg()
    sample = mm.data.make_sample([160, 120, 97], [5, 5, 5], img_tokens=37, img_dim=768, seed=4)
    ni = sample["net_input"]
    model.eval()
    with torch.no_grad():
        eo = model.encoder.forward_torchscript(ni)
        beam = 2
        eo = model.encoder.reorder_encoder_out(eo, torch.arange(3, device="cuda").repeat_interleave(beam))
        g = torch.Generator().manual_seed(0)
        toks = torch.randint(4, 1004, (6, 12), generator=g).cuda()
        toks[:, 0] = 2
        inc = {}
        order_full = torch.arange(6, device="cuda")
        for t in range(12):
            if t == 5:   # hypotheses permuted within sentences and one sentence leaving the batch
                new = torch.tensor([1, 0, 5, 4], device="cuda")
                model.reorder_incremental_state(inc, new)
                eo = model.reorder_encoder_out(eo, new)
                toks = toks[new]
            lg_inc, _ = model.decoder(toks[:, :t + 1], encoder_out=eo, incremental_state=inc)
            lg_full, _ = model.decoder(toks[:, :t + 1], encoder_out=eo)
            assert lg_inc.shape == (toks.shape[0], 1, 1004)
            assert _rel(lg_inc[:, 0], lg_full[:, -1]) < 1e-2, t
            lp = model.get_normalized_probs((lg_inc, None), log_probs=True)
            assert torch.allclose(lp.exp().sum(-1), torch.ones_like(lp[..., 0]), atol=1e-4)
    del order_full


def test_update_freq_accumulation_matches_union(tmp_path):
    """--update-freq 2: one update from two micro-batches; the gradient equals the union batch's
    gradient.  The union pads the second batch to a longer length, so GEMM accumulation order and
    fp16 rounding differ and FFN units within rounding of 0 switch ReLU sides:
    1e-2, the model-parity gradient tolerance.  Same-shape equality (accumulated vs DP-reduced)
    is checked at 1e-3 in test_gpu_dp.py."""
    mm = pkg()
    cfg = mm.default_cfg(**R.no_dropout(R.tiny_config(conv_channels=256)))
    samples = [mm.data.make_sample(L, T, img_tokens=37, img_dim=768, seed=s)
               for s, (L, T) in enumerate((([120, 90], [30, 22]), ([100, 77, 60], [25, 20, 15])))]
    grads = {}
    for name, uf in (("accum", 2), ("union", 1)):
        model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=5)
        tr = mm.trainer.Trainer(model, lr=1e-4, update_freq=uf, init_scale=8.0)
        tr.opt.defer = False
        if uf == 2:
            bs = [mm.runtime.prepare_batch(s, cfg, "cuda") for s in samples]
        else:
            items = []
            for s in samples:
                ni = s["net_input"]
                for b in range(ni["src_tokens"].shape[0]):
                    L = int(ni["src_lengths"][b])
                    items.append({"index": len(items), "source": ni["src_tokens"][b, :L], "target": s["target"][b][s["target"][b] != 1],
                                  "img": ni["imgs_list"][0][b]})
            bs = [mm.runtime.prepare_batch(mm.data.collater(items), cfg, "cuda")]
        log = tr.train_step(bs)
        torch.cuda.synchronize()
        assert not tr.opt.stats()["overflow"]
        grads[name] = (model.params.grad.float().cpu(), float(log[2]))
    assert grads["accum"][1] == grads["union"][1]
    assert _rel(grads["accum"][0], grads["union"][0]) < 1e-2


def test_cli_save_dir_checkpoint_and_restore(tmp_path, capsys):
    """--save-dir writes checkpoint_last.pt (fairseq keys, optimizer state, num_updates);
    a second run restores it and continues the update count (fairseq --restore-file)."""
    a = _args(tmp_path)
    y = a.multimodal_translation_config_yaml
    sd = tmp_path / "ckpt"
    base = (f"/d --task multimodal_speech_to_speech --arch mm_s2ut_transformer --criterion speech_to_unit "
            f"--target-is-code --target-code-size 1000 --share-decoder-input-output-embed --fp16 "
            f"--multimodal-translation-config-yaml {y} {TINY} --max-tokens 6000 --log-interval 2 "
            f"--warmup-updates 4 --lr 1e-3 --synthetic --save-dir {sd} --update-freq 2")
    assert pkg("cli").main((base + " --max-update 2").split()) == 0
    with torch.serialization.safe_globals([__import__("argparse").Namespace]):
        ck = torch.load(sd / "checkpoint_last.pt", map_location="cpu", weights_only=True)
    assert "encoder.transformer_layers.0.fc1.weight" in ck["model"]
    assert set(ck["last_optimizer_state"]) >= {"master", "exp_avg", "exp_avg_sq", "ost", "loss_scale"}
    n1 = ck["extra_state"]["num_updates"]
    assert n1 == 2 and ck["optimizer_history"][-1]["num_updates"] == 2   # fairseq num_updates: overflow skips excluded
    assert ck["extra_state"]["train_iterator"]["epoch"] >= 1 and ck["extra_state"]["train_iterator"]["iterations_in_epoch"] >= 2
    assert pkg("cli").main((base + " --max-update 4").split()) == 0
    recs = [json.loads(l) for l in capsys.readouterr().out.splitlines() if l.startswith("{")]
    assert recs[-1]["num_updates"] == 4
    with torch.serialization.safe_globals([__import__("argparse").Namespace]):
        ck2 = torch.load(sd / "checkpoint_last.pt", map_location="cpu", weights_only=True)
    assert ck2["extra_state"]["num_updates"] == 4


def test_cli_trains_on_manifest_with_multitask(tmp_path, capsys):
    """The reference recipe's --multitask-config-yaml (textless/1_train.sh:119): per-task dict.txt +
    {split}.tsv text targets, a transformer head on an encoder layer and CTC heads on encoder and
    decoder states, trained with the on-disk manifest path; the model's state carries the heads
    under fairseq's ``{task}_decoder.*`` names."""
    from manifest_corpus import write_corpus
    d = tmp_path / "data"
    d.mkdir()
    c = write_corpus(str(d), frames=(150, 97, 200, 61, 88, 131, 45, 170), di=768, ti=12)
    letters = "abcdefghij"
    mtd = tmp_path / "letters"
    mtd.mkdir()
    (mtd / "dict.txt").write_text("".join(f"{ch} 1\n" for ch in letters))
    rng = __import__("numpy").random.default_rng(0)
    rows = ["id\ttgt_text"] + [f"utt{k}\t{' '.join(rng.choice(list(letters), max(2, T // 20)))}"
                               for k, T in enumerate(c["frames"])]
    (mtd / "train.tsv").write_text("\n".join(rows) + "\n")
    mt = tmp_path / "config_multitask.yaml"
    mt.write_text(f"source_letter:\n  decoder_type: transformer\n  dict: {mtd}/dict.txt\n  data: {mtd}\n"
                  f"  encoder_layer: 2\n  loss_weight: 8.0\n  decoder_args:\n    decoder_layers: 1\n"
                  f"target_ctc:\n  decoder_type: ctc\n  dict: {mtd}/dict.txt\n  data: {mtd}\n  encoder_layer: 1\n"
                  f"  loss_weight: 1.0\ndecoder_ctc:\n  decoder_type: ctc\n  dict: {mtd}/dict.txt\n  data: {mtd}\n"
                  f"  decoder_layer: 2\n  loss_weight: 1.6\n")
    y = tmp_path / "mm.yaml"
    y.write_text(FUSION_YAML.replace('["/feats/vit_base_patch16_384"]', f'["{c["feat_dir"]}"]'))
    sd = tmp_path / "ck"
    argv = (f"{d} --task multimodal_speech_to_speech --arch mm_s2ut_transformer --criterion speech_to_unit "
            f"--config-yaml config.yaml --target-is-code --target-code-size 1000 --multitask-config-yaml {mt} "
            f"--share-decoder-input-output-embed --fp16 --multimodal-translation-config-yaml {y} {TINY} "
            f"--max-update 4 --max-tokens 600 --log-interval 4 --warmup-updates 4 --lr 1e-3 --save-dir {sd}").split()
    assert pkg("cli").main(argv) == 0
    recs = [json.loads(l) for l in capsys.readouterr().out.splitlines() if l.startswith("{")]
    assert [r["num_updates"] for r in recs] == [4] and recs[0]["loss"] > 0
    with torch.serialization.safe_globals([__import__("argparse").Namespace]):
        ck = torch.load(sd / "checkpoint_last.pt", map_location="cpu", weights_only=True)
    for k in ("source_letter_decoder.layers.0.encoder_attn.k_proj.weight", "source_letter_decoder.embed_tokens.weight",
              "target_ctc_decoder.proj.weight", "decoder_ctc_decoder.proj.bias"):
        assert k in ck["model"], k
    assert tuple(ck["model"]["source_letter_decoder.layers.0.encoder_attn.k_proj.weight"].shape) == (256, 256)


FUSION_NODROP = FUSION_YAML.replace("SA_image_dropout: 0.1", "SA_image_dropout: 0.0")


def _rel_all(ga, gb, names):
    num = sum(float((ga[n].float() - gb[n].float()).norm() ** 2) for n in names)
    den = sum(float(gb[n].float().norm() ** 2) for n in names)
    return (num / max(den, 1e-30)) ** 0.5


def test_fairseq_dropin_trains_like_native(monkeypatch, tmp_path):
    """fairseq-train's call sequence (stub fairseq restating its behaviour,
    tests/fairseq_stub.py) drives setup_task -> load_dataset -> build_model -> build_criterion ->
    criterion(model, sample) -> backward through the adapter.  With the stub's built-in
    speech_to_unit (the reference's criterion: model(**net_input, return_all_hiddens=True), then
    compute_loss(model, [net_output], sample) -> get_normalized_probs -> label_smoothed_nll_loss
    in torch fp32) the loss equals the native path's to 1e-5 and the per-parameter gradients to
    5e-3 (the two LS-CE implementations round dlogits to fp16 differently); through the adapter's
    own alias criterion (HIP LS-CE) both are bit-identical to the native path.  Dropout is on
    (p = 0.1 everywhere); each run restarts the dropout stream from the same seed."""
    import fairseq_stub
    fs, regs, args, c, _ = fairseq_stub.dropin_setup(monkeypatch, tmp_path, FUSION_NODROP)
    P = pkg("plugins")
    task = fs.tasks.setup_task(args)
    task.load_dataset("train")
    model = task.build_model(args).half()          # fairseq Trainer: model.half() for --fp16
    crit = task.build_criterion(args)
    alias = regs["criterion"]["speech_to_unit_v2"].build_criterion(args, task)
    batches = task.get_batch_iterator(task.dataset("train"), max_tokens=450, max_positions=task.max_positions())
    sample = fs.utils.apply_half(fs.utils.move_to_cuda(batches[0]))
    net = model.impl.net
    names = [n for n, _ in model.named_parameters()]
    model.train()
    runs = {}
    for kind in ("fairseq", "alias", "native", "at_end"):
        model.zero_grad(set_to_none=True)
        net.drop.reset(7)
        if kind == "at_end":
            # the loss-linked bridge: torch.autograd.grad over the parameters works
            model.grad_release = "at_end"
            loss, ss, log = alias(model, sample)
            grads = torch.autograd.grad(loss, [p for _, p in model.named_parameters()])
            model.grad_release = "per_group"
            torch.cuda.synchronize()
            g = {n: gr.clone() for (n, _), gr in zip(model.named_parameters(), grads)}
        elif kind == "native":
            net.params.grad.zero_()                # as the native Trainer does per micro-batch
            loss, ss, log = P.SpeechToUnitCriterion(task.impl, 0.2)(model.impl, sample)
            loss.backward()
            torch.cuda.synchronize()
            # every fairseq parameter is a view of the flat buffer (packed in_proj included): its
            # gradient is the same span of the flat gradient
            base = net.params.flat.data_ptr()
            g = {n: net.params.grad[(p.data_ptr() - base) // 2:][:p.numel()].view(p.shape).clone()
                 for n, p in model.named_parameters()}
        else:
            loss, ss, log = (crit if kind == "fairseq" else alias)(model, sample)
            loss.backward()
            torch.cuda.synchronize()
            g = {n: p.grad.clone() for n, p in model.named_parameters()}
        assert ss == sample["ntokens"] and log["nsentences"] == sample["target"].size(0)
        runs[kind] = (float(loss), g)
    ln, gn = runs["native"]
    la, ga = runs["alias"]
    lf, gf = runs["fairseq"]
    assert la == ln and all(torch.equal(ga[n], gn[n]) for n in names)
    le, ge = runs["at_end"]
    assert le == ln and all(torch.equal(ge[n], gn[n]) for n in names)
    assert abs(lf - ln) / abs(ln) < 1e-5, (lf, ln)
    assert _rel_all(gf, gn, names) < 5e-3
    fusion = [n for n in names if n.startswith("encoder.multimodal_attns.0.") and n.endswith("weight")]
    assert fusion
    for n in ["encoder.subsample.conv_layers.0.weight", "decoder.embed_tokens.weight"] + fusion:
        assert _rel_all(gf, gn, [n]) < 1e-2, n


def test_fairseq_dropin_multitask_ctc_matches_native(monkeypatch, tmp_path):
    """The reference recipe's multitask head through the drop-in: fairseq's own CTC decoder
    (stub CTCDecoder = Linear) reads extra["encoder_states"][0] from the HIP model's forward and
    the stub's MultitaskCriterion / CtcCriterion compute its loss in torch; the gradient it puts on
    the encoder state enters the hand-written backward.  Against the native path (HIP CTC head in
    the flat buffer, same weights): total loss to 1e-3, encoder gradients to 1e-2."""
    import fairseq_stub
    fs, regs, args, c, _ = fairseq_stub.dropin_setup(monkeypatch, tmp_path, FUSION_NODROP, multitask=True,
                                                     extra="--dropout 0 --attention-dropout 0 --relu-dropout 0")
    P = pkg("plugins")
    task = fs.tasks.setup_task(args)
    task.load_dataset("train")
    model = task.build_model(args).half()
    crit = task.build_criterion(args)
    native = P.MM_S2UTTransformerModel.build_model(args, task.impl)
    sd = {k: v for k, v in model.state_dict().items()}
    native.load_state_dict({k: v for k, v in sd.items() if k in native.net.params.offsets or k in native.net.params.unused})
    batches = task.get_batch_iterator(task.dataset("train"), max_tokens=450, max_positions=task.max_positions())
    sample = fs.utils.apply_half(fs.utils.move_to_cuda(batches[0]))
    model.train()
    native.train()
    loss_f, _, log = crit(model, sample)
    loss_f.backward()
    loss_n, _, logn = P.SpeechToUnitCriterion(task.impl, 0.2)(native, sample)
    loss_n.backward()
    torch.cuda.synchronize()
    assert "target_ctc" in log["multitask"] and float(log["multitask"]["target_ctc"]["loss"]) > 0
    assert abs(float(loss_f) - float(loss_n)) / abs(float(loss_n)) < 1e-3
    gf = {n: p.grad for n, p in model.named_parameters()}
    gn = {n: native.net.params.g[n] for n in native.net.params.offsets}
    enc = [n for n in gn if n.startswith("encoder.transformer_layers.0.")]
    assert _rel_all(gf, gn, enc) < 1e-2
    assert _rel_all(gf, gn, ["target_ctc_decoder.proj.weight"]) < 1e-2
    # the head's gradient reached the encoder: without it layer 0 would see only the main loss
    assert float(gf["encoder.transformer_layers.0.fc1.weight"].float().norm()) > 0
