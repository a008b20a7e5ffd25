"""Plugin surface (task / arch / criterion names, flags, fusion YAML) and the fairseq adapter.

fairseq is not importable here: the adapter is checked against a stub registry that mimics the
decorator API of fairseq.tasks / fairseq.models / fairseq.criterions.
"""
import sys  # noqa: F401
import types

import numpy as np

import pytest
import torch

from conftest import pkg

CANONICAL = (  # scripts/textless/1_train.sh:105-125 (paths replaced)
    "/data --distributed-world-size 1 --tensorboard-logdir /tmp/tb --config-yaml config.yaml "
    "--task multimodal_speech_to_speech --target-is-code --target-code-size 1000 --vocoder code_hifigan "
    "--criterion speech_to_unit --label-smoothing 0.2 --arch mm_s2ut_transformer "
    "--share-decoder-input-output-embed --dropout 0.1 --attention-dropout 0.1 --relu-dropout 0.1 "
    "--train-subset train --valid-subset valid --save-dir /tmp/ck --lr 0.0005 --lr-scheduler inverse_sqrt "
    "--warmup-init-lr 1e-7 --warmup-updates 10000 --optimizer adam --adam-betas (0.9,0.98) "
    "--clip-norm 10.0 --max-update 100 --max-tokens 40000 --max-target-positions 3000 --update-freq 1 "
    "--required-batch-size-multiple 1 --multitask-config-yaml config_multitask.yaml "
    "--multimodal-translation-config-yaml {yaml} --encoder-embed-dim 768 --encoder-ffn-embed-dim 3072 "
    "--gen-subset test --user-dir mm_s2ut --seed 1 --fp16 --num-workers 8")

# the shipped fusion YAML's effective values (mm_s2ut/config/multimodal_s2ut_transformer.yaml)
FUSION_YAML = """
SA_image_dropout: 0.1
SA_text_dropout: 0.0
SA_attention_dropout: 0.1
image_pre_norm: True
is_fusion_top: True
image_feat_path: ["/feats/vit_base_patch16_384"]
image_feat_dim: [768]
flickr30k_root: /flickr30k
load_visual_extractor_type: null
load_visual_extractor: null
modality_dropout: -0.5
audio_dropout: -0.5
multimodal_attention_type: multimodal_attention
use_selective_gate: True
is_merge_text_img: False
"""


def _plugins():
    return pkg("plugins")


def _args(tmp_path, extra=""):
    y = tmp_path / "mm.yaml"
    y.write_text(FUSION_YAML)
    mt = tmp_path / "config_multitask.yaml"     # the recipe's multitask config, here with no tasks
    mt.write_text("{}\n")
    cmd = CANONICAL.format(yaml=y).replace("config_multitask.yaml", str(mt))
    return _plugins().build_parser().parse_args((cmd + extra).split())


def test_registry_names():
    R = _plugins().REGISTRY
    assert "multimodal_speech_to_speech" in R["task"]
    assert "mm_s2ut_transformer" in R["model"] and "mm_s2ut_transformer" in R["arch"]
    for c in ("speech_to_unit", "speech_to_speech", "speech_to_unit_v2"):
        assert c in R["criterion"]


def test_canonical_command_gives_base_config(tmp_path):
    P = _plugins()
    a = _args(tmp_path)
    task = P.REGISTRY["task"][a.task].setup_task(a)
    cfg = P.cfg_from_args(a, task.multimodal_translation_config, task.vocab_size)
    assert cfg == pkg("model").default_cfg()
    assert task.vocab_size == 1004 and task.padding_idx == 1 and task.eos == 2


def test_arch_defaults_and_overrides(tmp_path):
    P = _plugins()
    a = _args(tmp_path, " --encoder-layers 2 --decoder-layers 2 --decoder-embed-dim 768")
    task = P.MultiModalSpeechToSpeechTask(a)
    cfg = P.cfg_from_args(a, task.multimodal_translation_config)
    assert cfg["encoder_layers"] == 2 and cfg["decoder_layers"] == 2
    assert cfg["decoder_ffn_embed_dim"] == 3072  # follows encoder_ffn_embed_dim (arch default)
    b = P.build_parser().parse_args(["/d", "--fp16", "--share-decoder-input-output-embed"])
    cfgb = P.cfg_from_args(b)
    assert cfgb["encoder_embed_dim"] == 512 and cfgb["max_target_positions"] == 1024
    assert cfgb["fusion"] is False


def test_unsupported_options_fail_loudly(tmp_path):
    P = _plugins()
    a = P.build_parser().parse_args(["/d", "--fp16"])  # no --share-decoder-input-output-embed
    with pytest.raises(NotImplementedError, match="share-decoder"):
        P.cfg_from_args(a)
    y = tmp_path / "sel.yaml"
    y.write_text(FUSION_YAML.replace("multimodal_attention_type: multimodal_attention",
                                     "multimodal_attention_type: merge_attention"))
    fus = P.load_fusion_yaml(str(y))
    a = P.build_parser().parse_args(["/d", "--fp16", "--share-decoder-input-output-embed"])
    with pytest.raises(NotImplementedError, match="merge_attention"):
        P.cfg_from_args(a, fus)
    y.write_text(FUSION_YAML.replace("image_feat_dim: [768]", "image_feat_dim: [256, 768]"))
    with pytest.raises(NotImplementedError, match="one image-feature type"):
        P.cfg_from_args(a, P.load_fusion_yaml(str(y)))
    with pytest.raises(NotImplementedError, match="pretrained"):
        P.MultiModalSpeechToSpeechTask(P.build_parser().parse_args(
            ["/d", "--fp16", "--wav2vec2-model-dir", "/w2v"]))


def test_selective_attention_yaml(tmp_path):
    P = _plugins()
    y = tmp_path / "sel.yaml"
    y.write_text(FUSION_YAML.replace("multimodal_attention_type: multimodal_attention",
                                     "multimodal_attention_type: selective_attention")
                 .replace("use_selective_gate: True", "use_selective_gate: False"))
    a = P.build_parser().parse_args(["/d", "--fp16", "--share-decoder-input-output-embed"])
    cfg = P.cfg_from_args(a, P.load_fusion_yaml(str(y)))
    assert cfg["multimodal_attention_type"] == "selective_attention"
    assert cfg["use_selective_gate"] is False and cfg["fusion"] is True


def test_qformer_yaml(tmp_path):
    """multimodal_extractor_type: q_former (mm_s2s_transformer.py:194-209): with a visual extractor
    configured the QFormer runs on the image features (its parameters are trained); without one the
    reference builds it and never calls it (:475), so its parameters are kept but unused."""
    P, mm = _plugins(), pkg()
    a = P.build_parser().parse_args(["/d", "--fp16", "--share-decoder-input-output-embed", "--encoder-embed-dim", "768"])
    base = FUSION_YAML + "multimodal_extractor_type: q_former\nnum_queries: 16\nnum_query_layers: 2\n"
    for extractor, active in (("vit_huggingface", True), ("null", False)):
        y = tmp_path / f"qf_{extractor}.yaml"
        y.write_text(base.replace("load_visual_extractor_type: null", f"load_visual_extractor_type: {extractor}"))
        cfg = P.cfg_from_args(a, P.load_fusion_yaml(str(y)))
        specs, unused = mm.param_specs(cfg)
        used = {n for n, _ in specs if n.startswith("encoder.q_former.")}
        idle = {n for n, _ in unused if n.startswith("encoder.q_former.")}
        assert cfg["num_queries"] == 16 and cfg["num_query_layers"] == 2 and cfg["num_multimodal_layers"] == 2
        assert (cfg["multimodal_extractor_type"] == "q_former") == active
        assert bool(used) == active and bool(idle) == (not active)
        assert dict(specs + unused)["encoder.q_former.query_embedding"] == (1, 16, 768)
        assert len(used | idle) == 1 + 4 * 18   # query embedding + 18 tensors per layer


def test_cli_rejects_non_fp16_and_missing_data():
    cli = pkg("cli")
    with pytest.raises(SystemExit, match="fp16"):
        cli.main(["/d", "--share-decoder-input-output-embed"])
    with pytest.raises(SystemExit, match="DATA"):
        cli.main(["--fp16", "--share-decoder-input-output-embed"])
    with pytest.raises(SystemExit, match="unknown criterion"):
        cli.main(["/d", "--fp16", "--criterion", "cross_entropy", "--synthetic"])


def test_fairseq_adapter_registers_reference_names(monkeypatch):
    import fairseq_stub
    fs, regs = fairseq_stub.install(monkeypatch)
    task, model, crits, _ = pkg("fairseq_adapter").register(fs)
    assert regs["task"]["multimodal_speech_to_speech"] is task
    assert regs["model"]["mm_s2ut_transformer"] is model
    assert regs["arch"]["mm_s2ut_transformer"] is model
    # fairseq's built-in speech_to_unit keeps its name; the free aliases are ours
    assert regs["criterion"]["speech_to_unit"].__name__ == "SpeechToUnit"    # the stub's built-in
    assert set(crits) == {"speech_to_speech", "speech_to_unit_v2"}
    ns = types.SimpleNamespace()
    regs["arch_cfg"]["mm_s2ut_transformer"](ns)
    assert ns.encoder_embed_dim == 512 and ns.decoder_layers == 6 and ns.conv_channels == 1024


def test_fairseq_dropin_task_dataset_model_cpu(monkeypatch, tmp_path):
    """fairseq-train's call sequence against the adapter, up to the model's forward (which needs
    the GPU; tests/test_gpu_plugins.py runs the rest): setup_task -> load_dataset -> batches ->
    build_model -> build_criterion, with the reference's contracts checked at each step
    (criterions/speech_to_speech_criterion.py:56,73-76; tasks/speech_to_speech.py:83-123)."""
    import fairseq_stub
    fs, regs, args, c, _ = fairseq_stub.dropin_setup(monkeypatch, tmp_path, FUSION_YAML, multitask=True)
    base = fs.tasks.LegacyFairseqTask(args)     # the stub base restates fairseq's abstract members
    with pytest.raises(NotImplementedError):
        base.load_dataset("train")
    with pytest.raises(NotImplementedError):
        base.target_dictionary
    task = fs.tasks.setup_task(args)
    assert len(task.target_dictionary) == 1004 and task.target_dictionary.pad() == 1
    assert task.source_dictionary is None
    assert set(task.multitask_tasks) == {"target_ctc"}
    mt = task.multitask_tasks["target_ctc"]
    assert (mt.args.input_from, mt.args.input_layer, mt.args.decoder_type) == ("encoder", 0, "ctc")
    ds = task.load_dataset("train")
    assert task.dataset("train") is ds and len(ds) == 6
    batches = task.get_batch_iterator(ds, max_tokens=450, max_positions=task.max_positions())
    seen = []
    for sample in batches:
        ni = sample["net_input"]
        ids = sample["id"].tolist()
        seen += ids
        assert ni["src_tokens"] is None and ni["src_lengths"].tolist() == sorted(ni["src_lengths"].tolist(), reverse=True)
        # the waveforms travel as the int32 bit patterns of the fp32 samples (apply_half-proof)
        assert ni["src_waves"].dtype == torch.int32
        off = ni["src_wave_offsets"].tolist()
        for j, i in enumerate(ids):
            w = ni["src_waves"][off[j]:off[j + 1]].view(torch.float32).numpy()
            assert np.array_equal(w, c["waves"][i])
        assert fs.utils.apply_half(sample)["net_input"]["src_waves"].dtype == torch.int32
        assert ni["imgs_list"][0].shape[1:] == (12, 768) and ni["img_masks_list"][0].dtype == torch.bool
        assert sample["target"][:, -1].tolist() == [2 if t == sample["target"].shape[1] else 1
                                                    for t in sample["target_lengths"].tolist()]
        assert set(sample["multitask"]) == {"target_ctc"}
        assert sample["multitask"]["target_ctc"]["target"].shape[0] == len(ids)
    assert sorted(seen) == list(range(6))
    model = task.build_model(args)
    # the reference model's state-dict keys (fairseq module tree), every parameter a view of the
    # flat HIP buffer; the multitask head is fairseq's own module under {task}_decoder.*
    sd = model.state_dict()
    ref_keys = set(model.impl.net.params.state_dict())
    assert ref_keys <= set(sd) and "decoder.output_projection.weight" in sd
    assert "encoder.proj_768_to_512.weight" in sd and "target_ctc_decoder.proj.weight" in sd
    assert "flat" not in sd
    flat = model.impl.net.params.flat
    lo, hi = flat.data_ptr(), flat.data_ptr() + 2 * flat.numel()
    named = dict(model.named_parameters())
    assert all(lo <= p.data_ptr() < hi for n, p in named.items() if not n.startswith("target_ctc_decoder"))
    assert model.get_parameter("decoder.output_projection.weight") is model.get_parameter("decoder.embed_tokens.weight")
    assert set(model.multitask_decoders) == {"target_ctc"}
    # a checkpoint round trip through the fairseq key names writes the flat buffer
    sd2 = {k: v.clone() for k, v in sd.items()}
    sd2["encoder.layer_norm.weight"].fill_(0.5)
    model.load_state_dict(sd2, strict=True)
    assert torch.all(model.impl.net.params.p["encoder.layer_norm.weight"] == 0.5)
    # get_normalized_probs on the criterion's one-element list (compute_loss(model, [net_output]))
    lg = torch.randn(2, 3, 1004)
    lp = model.get_normalized_probs([lg], log_probs=True)
    assert torch.allclose(lp.exp().sum(-1), torch.ones(2, 3), atol=1e-5)
    crit = task.build_criterion(args)
    assert type(crit).__name__ == "SpeechToUnit" and crit.eps == 0.2 and set(crit.multitask_criterion) == {"target_ctc"}


def _reducer_worker(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        par = pkg("parallel")
        r, w, _ = par.init_from_env(backend="gloo")
        n = 1000
        g = torch.arange(n, dtype=torch.float32) * (r + 1)
        # 256-element buckets; host tensors: the DDP pre-division by world as a host op
        red = par.GradAllReducer(g, bucket_mb=256 * 4 / 2 ** 20, prescale=lambda b, a: b.mul_(a))
        assert len(red.bounds) == 4
        for upto in (100, 300, 600, 1000):  # layer completion offsets
            red.ready(upto)
        launched_before_finish = red.next
        red.finish()
        s = torch.tensor([1.0 + r, 10.0 * (r + 1)])
        par.all_reduce_scalars(s)
        q.put((r, launched_before_finish, torch.equal(g, torch.arange(n, dtype=torch.float32) * 1.5),
               s.tolist()))
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e), None))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_allreducer_gloo_world2():
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r, launched, ok, scal in res:
        assert launched == 4, (r, launched, ok)  # every bucket launched during the "backward"
        assert ok is True
        assert scal == [3.0, 30.0]


def test_multitask_config_and_text_targets(tmp_path):
    """fairseq MultitaskConfig / TextTargetMultitaskData restatement: input_from / input_layer,
    defaults, dict.txt, eos appended except for CTC, collater (eos-first prev_output_tokens)."""
    MT = pkg("multitask")
    d = tmp_path / "letters"
    d.mkdir()
    (d / "dict.txt").write_text("a 10\nb 7\nc 3\n")
    (d / "train.tsv").write_text("id\ttgt_text\nu1\ta b c\nu2\tc a\n")
    y = tmp_path / "mt.yaml"
    y.write_text(f"src_letter:\n  decoder_type: transformer\n  dict: {d}/dict.txt\n  data: {d}\n  encoder_layer: 6\n"
                 f"  loss_weight: 8.0\nctc_tgt:\n  decoder_type: ctc\n  dict: {d}/dict.txt\n  data: {d}\n"
                 f"  decoder_layer: 3\n  loss_weight: 1.6\n")
    raw = MT.load_multitask_config(str(y))
    assert list(raw) == ["src_letter", "ctc_tgt"]
    assert MT.input_spec(raw["src_letter"]) == ("encoder", 5)
    assert MT.input_spec(raw["ctc_tgt"]) == ("decoder", 2)
    assert MT.input_spec({"decoder_type": "ctc"}) == ("encoder", -1)
    dct = MT.Dictionary.load(raw["src_letter"]["dict"])
    assert len(dct) == 7 and dct.index["a"] == 4
    cfg = pkg().default_cfg()
    t = MT.task_model_cfg("src_letter", raw["src_letter"], dct, cfg)
    assert (t["d"], t["H"], t["F"], t["L"], t["dropout"], t["layer"]) == (256, 4, 2048, 2, 0.3, 5)
    c = MT.task_model_cfg("ctc_tgt", raw["ctc_tgt"], dct, cfg)
    assert c["blank"] == 0 and c["zero_infinity"] and c["layer"] == 2
    tx = MT.TextTargetMultitaskData(str(d), "train", dct, "transformer")
    assert tx.get("u1").tolist() == [4, 5, 6, 2]
    assert MT.TextTargetMultitaskData(str(d), "train", dct, "ctc").get("u2").tolist() == [6, 4]
    col = tx.collater([tx.get("u1"), tx.get("u2")])
    assert col["target"].tolist() == [[4, 5, 6, 2], [6, 4, 2, 1]]
    assert col["prev_output_tokens"].tolist() == [[2, 4, 5, 6], [2, 6, 4, 1]]
    assert col["target_lengths"].tolist() == [4, 3] and col["ntokens"] == 7
    # the heads enter the flat layout with fairseq's key names
    cfg["multitask"] = [t, c]
    names = [n for n, _ in pkg("model").param_specs(cfg)[0]]
    assert "src_letter_decoder.layers.1.encoder_attn.k_proj.weight" in names
    assert names.index("ctc_tgt_decoder.proj.weight") < names.index("decoder.layer_norm.weight")
    assert names.index("src_letter_decoder.embed_tokens.weight") < names.index("encoder.layer_norm.weight")
