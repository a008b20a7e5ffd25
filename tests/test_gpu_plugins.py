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
