"""CPU: pin the oracle's fairseq-S2T restatement (Conv1dSubsampler, sinusoidal positions, pre-LN
encoder/decoder layers, final LNs) against an INDEPENDENT implementation of the same fairseq
architecture: transformers' Speech2Text port (converted from fairseq S2T checkpoints).  fairseq
itself is absent from the container, so this is the strongest pin available for
rows A3–A5 / A10; the fusion rows are pinned by the reference itself (test_oracle_golden.py)."""
import pytest
import torch

from oracle import ref_model as R

transformers = pytest.importorskip("transformers")


def _hf_model(cfg):
    from transformers import Speech2TextConfig, Speech2TextModel
    c = Speech2TextConfig(
        vocab_size=cfg["vocab_size"], d_model=cfg["encoder_embed_dim"],
        encoder_layers=cfg["encoder_layers"], encoder_ffn_dim=cfg["encoder_ffn_embed_dim"],
        encoder_attention_heads=cfg["encoder_attention_heads"],
        decoder_layers=cfg["decoder_layers"], decoder_ffn_dim=cfg["decoder_ffn_embed_dim"],
        decoder_attention_heads=cfg["decoder_attention_heads"], activation_function="relu",
        scale_embedding=True, pad_token_id=1, bos_token_id=0, eos_token_id=2,
        num_conv_layers=2, conv_kernel_sizes=[5, 5], conv_channels=cfg["conv_channels"],
        input_feat_per_channel=80, input_channels=1, dropout=0.0, attention_dropout=0.0,
        activation_dropout=0.0, max_source_positions=600, max_target_positions=300)
    c._attn_implementation = "eager"
    return Speech2TextModel(c).double().eval()


def _load(hf, P):
    sd = {}
    for k, v in P.items():
        if k.startswith("encoder.subsample."):
            sd[k.replace("encoder.subsample.", "encoder.conv.")] = v
        elif k.startswith("encoder.transformer_layers."):
            sd[k.replace("encoder.transformer_layers.", "encoder.layers.")] = v
        elif k.startswith("encoder.layer_norm") or k.startswith("decoder."):
            sd[k] = v
    missing, _ = hf.load_state_dict({k: v.double() for k, v in sd.items()}, strict=False)
    assert all("embed_positions" in m for m in missing), missing


def test_encoder_decoder_match_speech2text_port():
    torch.manual_seed(0)
    cfg = R.no_dropout(R.tiny_config(fusion=False, conv_channels=128, vocab_size=40))
    P = R.init_params(cfg, seed=3, include_unused=False)
    hf = _hf_model(cfg)
    _load(hf, P)
    B, Ts = 3, 37
    lens = torch.tensor([37, 30, 21])
    x = torch.randn(B, Ts, 80, dtype=torch.float64)
    x[torch.arange(Ts)[None, :] >= lens[:, None]] = 0.0
    enc, pad, _ = R.encoder_forward(P, x, lens, cfg, dtype=torch.float64)
    am = (~R.lengths_to_padding_mask(lens, Ts)).long()
    hf_enc = hf.encoder(x, attention_mask=am).last_hidden_state          # B,T,C
    keep = ~pad
    torch.testing.assert_close(enc.transpose(0, 1)[keep], hf_enc[keep], rtol=1e-9, atol=1e-9)
    # decoder: prev_output_tokens with right padding
    Tt = 9
    prev = torch.randint(4, 40, (B, Tt))
    prev[:, 0] = 2
    tl = torch.tensor([9, 7, 4])
    prev[torch.arange(Tt)[None, :] >= tl[:, None]] = 1
    logits = R.decoder_forward(P, prev, enc, pad, cfg, dtype=torch.float64)
    hf_dec = hf.decoder(input_ids=prev, encoder_hidden_states=hf_enc,
                        encoder_attention_mask=am[:, ::4][:, :enc.shape[0]] * 0 + keep.long()
                        ).last_hidden_state
    ref_logits = hf_dec @ P["decoder.embed_tokens.weight"].double().t()
    tkeep = torch.arange(Tt)[None, :] < tl[:, None]
    torch.testing.assert_close(logits[tkeep], ref_logits[tkeep], rtol=1e-9, atol=1e-9)


def test_subsampler_lengths_known_answer():
    cfg = R.tiny_config(conv_channels=32, encoder_embed_dim=16)
    P = R.init_params(R.tiny_config(conv_channels=32, encoder_embed_dim=16, fusion=False,
                                    encoder_layers=0, decoder_layers=0), include_unused=False)
    for L in (1, 2, 3, 4, 5, 8, 9, 300, 1001):
        x = torch.randn(1, L, 80)
        y, out = R.conv1d_subsampler(P, x, torch.tensor([L]))
        exp = ((L - 1) // 2 + 1 - 1) // 2 + 1
        assert int(out) == exp == y.shape[0]
    del cfg


def test_sinusoidal_table_layout():
    t = R.sinusoidal_table(10, 8, padding_idx=1)
    assert torch.all(t[1] == 0)
    half = 4
    f = torch.exp(torch.arange(half, dtype=torch.float) * -(torch.log(torch.tensor(10000.0)) / (half - 1)))
    torch.testing.assert_close(t[5, :half], torch.sin(5 * f))
    torch.testing.assert_close(t[5, half:], torch.cos(5 * f))
    pos = R.make_positions(torch.tensor([[5, 6, 1, 1], [7, 8, 9, 1]]), 1)
    assert pos.tolist() == [[2, 3, 1, 1], [2, 3, 4, 1]]


def test_label_smoothed_ce_closed_form():
    torch.manual_seed(1)
    V, eps = 7, 0.2
    logits = torch.randn(2, 3, V, dtype=torch.float64)
    target = torch.tensor([[3, 1, 0], [6, 2, 1]])
    loss, nll = R.label_smoothed_nll_loss(logits, target, eps, ignore_index=1)
    lp = torch.log_softmax(logits, -1).view(-1, V)
    t = target.view(-1)
    keep = t != 1
    n = -lp[keep, t[keep]].sum()
    s = -lp[keep].sum()
    ei = eps / (V - 1)
    torch.testing.assert_close(loss, (1 - eps - ei) * n + ei * s)
    torch.testing.assert_close(nll, n)
