"""CPU: C-ABI library loads and exports every declared symbol; host-side logic (collater, batching,
parameter layout/state-dict names, fbank oracle cross-check, optimizer restatement)."""
import ctypes
import os
import re
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg
from oracle import ref_fbank as RF
from oracle import ref_model as R


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "mms2ut.h")).read()
    return sorted(set(re.findall(r"\b(mms2ut_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    mm = pkg()
    lib = mm._lib.load()
    syms = header_symbols()
    assert len(syms) > 30
    for s in syms:
        assert s in mm._lib.SIGNATURES, f"{s} declared in include/mms2ut.h but not bound in _lib.py"
        assert getattr(lib, s) is not None
    raw = ctypes.CDLL(mm._lib.LIB_PATH)
    for s in syms:
        getattr(raw, s)
    assert lib.mms2ut_version() == 1
    assert set(mm._lib.SIGNATURES) == set(syms)


def test_library_error_path_without_gpu():
    """A bad call fails loudly with a message (validation happens before any device work)."""
    mm = pkg()
    a = mm._lib.GemmArgs()
    a.M, a.N, a.K, a.batch, a.lda, a.ldb = 4, 4, 4, 1, 3, 8
    with pytest.raises(mm._lib.HipError, match="multiples of 8"):
        mm._lib.call("mms2ut_gemm_f16", ctypes.byref(a), None)
    b = mm._lib.GEMM_ARGS.pack(*[getattr(a, f) or 0 for f, _ in a._fields_])
    with pytest.raises(mm._lib.HipError, match="multiples of 8"):
        mm._lib.call("mms2ut_gemm_f16", b, None)


def test_gemm_args_pack_layout():
    """_lib.GEMM_ARGS / ATTN_ARGS (the struct-packed argument blocks kernels.gemm / _attn_args pass)
    have GemmArgs' / AttnArgs' layout: every field lands at its ctypes offset."""
    mm = pkg()
    for G, S in ((mm._lib.GemmArgs, mm._lib.GEMM_ARGS), (mm._lib.AttnArgs, mm._lib.ATTN_ARGS)):
        vals = [(i + 1) * (3 if t is not ctypes.c_float else 0.5) for i, (_, t) in enumerate(G._fields_)]
        g = G.from_buffer_copy(S.pack(*vals))
        assert [getattr(g, f) for f, _ in G._fields_] == vals, G


def test_param_layout_matches_reference_state_dict():
    mm = pkg()
    for cfg_o in (R.base_config(), R.tiny_config(image_feat_dim=768),
                  R.base_config(multimodal_attention_type="selective_attention"),
                  R.base_config(multimodal_extractor_type="q_former", num_queries=8, num_query_layers=2,
                                num_multimodal_layers=1, self_attention_first=False)):
        specs, unused = mm.param_specs(mm.default_cfg(**cfg_o))
        names = {n for n, _ in specs} | {n for n, _ in unused}
        ref = R.init_params(cfg_o, include_unused=True)
        assert names == set(ref), set(ref) ^ names
        shapes = dict(specs + unused)
        for k, v in ref.items():
            assert tuple(v.shape) == tuple(shapes[k]), k
    specs, unused = mm.param_specs(mm.default_cfg())
    n_used = sum(int(np.prod(s)) for _, s in specs)
    n_unused = sum(int(np.prod(s)) for _, s in unused)
    assert 149e6 < n_used < 152e6 and 13e6 < n_unused < 14e6   # ~164M total


def test_flat_layout_spans_contiguous():
    mm = pkg()
    ps = mm.model.ParamStore(mm.param_specs(mm.default_cfg())[0], "cpu")
    p = "encoder.transformer_layers.3.self_attn"
    qkv = ps.span(p + ".q_proj.weight", p + ".v_proj.weight")
    assert qkv.numel() == 3 * 768 * 768
    assert ps.span(p + ".q_proj.bias", p + ".v_proj.bias").numel() == 3 * 768
    for name, (off, shape, n) in ps.offsets.items():
        assert off % 8 == 0
    # all decoder layers' cross-attention K/V projections form one [L_d*2d, d] slab (one GEMM)
    L = mm.default_cfg()["decoder_layers"]
    f, t = "decoder.layers.0.encoder_attn", f"decoder.layers.{L - 1}.encoder_attn"
    assert ps.span(f + ".k_proj.weight", t + ".v_proj.weight").numel() == L * 2 * 768 * 768
    assert ps.span(f + ".k_proj.bias", t + ".v_proj.bias").numel() == L * 2 * 768
    l1 = "decoder.layers.1.encoder_attn"
    assert ps.offsets[l1 + ".k_proj.weight"][0] == ps.offsets[f + ".v_proj.weight"][0] + 768 * 768


def test_collater_contract():
    mm = pkg()
    s = mm.data.make_sample([30, 50, 40], [5, 9, 7], img_tokens=4, img_dim=8, img_mask=True)
    ni = s["net_input"]
    assert ni["src_lengths"].tolist() == [50, 40, 30]
    assert ni["src_tokens"].shape == (3, 50, 80)
    assert torch.all(ni["src_tokens"][2, 30:] == 0)
    assert s["target"][0, -1] == 2 and s["target"][2, 5:].eq(1).all()
    assert ni["prev_output_tokens"][0, 0] == 2
    assert torch.equal(ni["prev_output_tokens"][0, 1:], s["target"][0, :-1])
    assert s["ntokens"] == 21
    assert ni["imgs_list"][0].shape == (3, 4, 8) and ni["img_masks_list"][0].dtype == torch.bool
    assert s["id"].tolist() == [1, 2, 0]


def test_batch_by_size_max_tokens():
    mm = pkg()
    rng = np.random.default_rng(0)
    lens = mm.data.synth_lengths(5000, rng)
    assert lens.min() >= 150 and lens.max() <= 1000
    batches = mm.data.batch_by_size(lens, 40000)
    assert sorted(i for b in batches for i in b) == list(range(5000))
    for b in batches:
        assert len(b) * max(lens[b]) <= 40000


def test_prepare_batch_host_masks():
    mm = pkg()
    cfg = mm.default_cfg()
    s = mm.data.make_sample([93, 80, 61], [30, 25, 19], img_tokens=5, img_dim=768, img_mask=True)
    b = mm.runtime.prepare_batch(s, cfg, device="cpu")
    assert b.Te == 24 and b.enc_len32.tolist() == [24, 20, 16]
    assert b.tgt_mask.shape == (3, 32) and b.tgt_mask[2, 19:30].all() and not b.tgt_mask[0, :30].any()
    assert b.img_keymask.shape == (3, 8) and b.img_keymask[:, 5:].eq(0).all()
    assert b.n_src_frames == 234 and b.ntokens == 74


def test_fbank_oracle_vs_transformers_kaldi():
    """ref_fbank (restating torchaudio.compliance.kaldi.fbank) vs transformers.audio_utils'
    independent Kaldi-compatible implementation."""
    au = pytest.importorskip("transformers.audio_utils")
    rng = np.random.default_rng(0)
    for T in (1, 7, 150):
        w = RF.synth_wave(T, rng)
        a = RF.fbank(w)
        mf = au.mel_filter_bank(num_frequency_bins=257, num_mel_filters=80, min_frequency=20,
                                max_frequency=8000, sampling_rate=16000, norm=None, mel_scale="kaldi",
                                triangularize_in_mel_space=True)
        win = au.window_function(400, "povey", periodic=False)
        b = au.spectrogram(w, win, frame_length=400, hop_length=160, fft_length=512, power=2.0,
                           center=False, preemphasis=0.97, mel_filters=mf, log_mel="log",
                           mel_floor=1.192092955078125e-07, remove_dc_offset=True).T
        assert a.shape == b.shape == (T, 80)
        np.testing.assert_allclose(a, b, atol=2e-4, rtol=1e-5)


def test_fbank_known_answers():
    rng = np.random.default_rng(1)
    assert RF.num_frames(399) == 0 and RF.num_frames(400) == 1 and RF.num_frames(560) == 2
    # a pure tone puts its energy in the mel bin whose centre is nearest the tone
    n = 16000
    t = np.arange(n) / 16000.0
    w = (0.5 * np.sin(2 * np.pi * 1000.0 * t) * 2 ** 15).astype(np.float32)
    f = RF.fbank(w)
    banks = RF.mel_banks()
    centre = banks.argmax(1) * 16000 / 512
    assert abs(centre[f.mean(0).argmax()] - 1000.0) < 80.0
    c = RF.utterance_cmvn(f + rng.standard_normal(f.shape).astype(np.float32))
    np.testing.assert_allclose(c.mean(0), 0, atol=1e-4)
    np.testing.assert_allclose(c.std(0), 1, atol=1e-3)


def test_product_mel_banks_match_oracle():
    mm = pkg()
    np.testing.assert_array_equal(mm.frontend.mel_banks()[:, :256], RF.mel_banks())


def test_optimizer_restatement_adam_known_answer():
    p = torch.tensor([1.0, -2.0])
    g = torch.tensor([0.5, 0.25])
    m, v = torch.zeros(2), torch.zeros(2)
    R.adam_step(p, g, m, v, 1, lr=0.1)
    # first Adam step moves each coordinate by ~lr*sign(g)
    torch.testing.assert_close(p, torch.tensor([0.9, -2.1]), atol=1e-6, rtol=0)


def test_lr_schedule_inverse_sqrt():
    mm = pkg()

    class FakeParams:
        flat = torch.zeros(8, dtype=torch.float16)
        grad = torch.zeros(8, dtype=torch.float16)

    opt = mm.optim.FP16Adam(FakeParams(), lr=5e-4, warmup_updates=10000, warmup_init_lr=1e-7)
    assert abs(opt.get_lr() - 1e-7) < 1e-12
    opt.num_updates = 5000
    assert abs(opt.get_lr() - (1e-7 + 5000 * (5e-4 - 1e-7) / 10000)) < 1e-12
    opt.num_updates = 40000
    assert abs(opt.get_lr() - 5e-4 * (10000 / 40000) ** 0.5) < 1e-12
    assert opt.scale_window == 16384


def test_param_groups_tile_flat_buffer():
    """The deferred optimizer's forward-consumption groups tile the flat buffer."""
    mm = pkg()
    ps = mm.model.ParamStore(mm.param_specs(mm.default_cfg())[0], "cpu")
    g = ps.groups
    assert g[0][0] == "sub" and g[1][0] == "enc0" and g[-1][0] == "dec_ln"
    spans = sorted((a, b) for _, a, b in g)
    assert spans[0][0] == 0 and spans[-1][1] == ps.numel
    assert all(spans[i][1] == spans[i + 1][0] for i in range(len(spans) - 1))
    for name in ps.offsets:
        grp = ps.group_of(name)
        a, b = [(x, y) for n, x, y in g if n == grp][0]
        off, _, n = ps.offsets[name]
        assert a <= off and off + n <= b, name


def test_deal_batches_balanced_and_round_robin():
    """DP batch dealing: equal batch counts per rank; balanced groups pair batches of
    near-equal padded cost per update step; round-robin is fairseq's shuffled ShardedIterator."""
    D = pkg("data")
    corpus = D.SyntheticSpeechMulti30K(n_utts=3000, seed=1, with_images=False)
    batches = corpus.batches(40000)
    costs = [D.padded_cost([int(corpus.lengths[i]) for i in b]) for b in batches]
    for world in (1, 2, 8):
        bal = D.deal_batches(costs, world, seed=1, epoch=3)
        rr = D.deal_batches(costs, world, seed=1, epoch=3, balanced=False)
        assert len({len(m) for m in bal}) == 1 and len({len(m) for m in rr}) == 1
        assert len(bal[0]) == len(batches) // world == len(rr[0])
        flat = sorted(i for m in bal for i in m)
        assert len(set(flat)) == len(flat)                      # no batch dealt twice
        assert bal == D.deal_batches(costs, world, seed=1, epoch=3)   # deterministic per (seed, epoch)
        if world > 1:
            def eff(m):   # per-step DP efficiency: mean / max cost over the ranks (max sets the step time)
                c = np.array([[costs[m[r][s]] for r in range(world)] for s in range(len(m[0]))])
                return c.mean(1) / c.max(1)
            eb, er = eff(bal), eff(rr)
            assert eb.mean() >= er.mean() and np.median(eb) > 0.99
    # round-robin: the legacy permutation dealing
    order = np.random.RandomState(4).permutation(len(batches)).tolist()
    order = order[: len(order) // 2 * 2]
    assert D.deal_batches(costs, 2, seed=1, epoch=3, balanced=False) == [order[0::2], order[1::2]]


def test_bench_gpus_flag_launches_ranks(monkeypatch):
    """`bench.py --gpus N` starts N ranks itself (torch.distributed.run as a
    child process) when no launcher is around it, and fails loudly when a launcher's WORLD_SIZE
    disagrees with --gpus."""
    import argparse
    import subprocess
    import bench
    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("MMS2UT_DIST_BACKEND", "gloo")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "4"])
    with pytest.raises(SystemExit) as e:
        bench.launch_ranks(argparse.Namespace(gpus=2))
    assert e.value.code == 0 and len(calls) == 1
    cmd, env = calls[0]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and env["MASTER_ADDR"] == "127.0.0.1"
    assert cmd[-4:] == [bench.__file__.replace(".pyc", ".py"), "--gpus", "2", "--steps", "4"][-4:]
    # one GPU: nothing to launch
    assert bench.launch_ranks(argparse.Namespace(gpus=1)) is None
    # under a launcher, the sizes must agree
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.launch_ranks(argparse.Namespace(gpus=8))
    assert bench.launch_ranks(argparse.Namespace(gpus=4)) is None
    # RCCL needs a GPU per rank
    monkeypatch.delenv("WORLD_SIZE")
    monkeypatch.delenv("MMS2UT_DIST_BACKEND")
    with pytest.raises(SystemExit, match="visible GPUs"):
        bench.launch_ranks(argparse.Namespace(gpus=2))


def test_checkpoint_interchange_fairseq_layout(tmp_path):
    """our checkpoint carries fairseq's top-level layout (model, last_optimizer_state
    with loss_scale, optimizer_history, extra_state with the train iterator, args as an
    argparse.Namespace) and round-trips exactly; a fairseq-written checkpoint (FP16Optimizer state
    in fairseq's own layout) restores the weights, re-derives the fp32 master from them, starts
    fresh Adam moments and keeps num_updates and the loss scale."""
    import argparse
    mm = pkg()
    K = mm.kernels
    cfg = mm.default_cfg(**R.no_dropout(R.tiny_config(conv_channels=256)))
    model = mm.MMS2UTModel(cfg, device="cpu").init_params(seed=2)
    tr = mm.trainer.Trainer(model, lr=1e-3)
    tr.opt.ost[K.OST_STEP] = 5.0
    tr.opt.ost[K.OST_LOSS_SCALE] = 32.0
    tr.opt.exp_avg.fill_(0.25)
    tr.position = {"epoch": 3, "iterations_in_epoch": 7}
    st = tr.state_dict()
    st["args"] = argparse.Namespace(arch="mm_s2ut_transformer", seed=1)
    path = tmp_path / "checkpoint_last.pt"
    torch.save(st, path)
    with torch.serialization.safe_globals([argparse.Namespace]):
        ck = torch.load(path, map_location="cpu", weights_only=True)
    assert ck["optimizer_history"][-1]["num_updates"] == 5 and ck["extra_state"]["num_updates"] == 5
    assert ck["extra_state"]["train_iterator"] == {"epoch": 3, "iterations_in_epoch": 7, "shuffle": True}
    assert ck["last_optimizer_state"]["loss_scale"] == 32.0 and ck["args"].arch == "mm_s2ut_transformer"
    model2 = mm.MMS2UTModel(cfg, device="cpu").init_params(seed=9)
    tr2 = mm.trainer.Trainer(model2, lr=1e-3)
    tr2.load_state_dict(ck)
    assert torch.equal(model2.params.flat, model.params.flat) and torch.all(tr2.opt.exp_avg == 0.25)
    assert tr2.completed_updates() == 5
    # fairseq's own FP16Optimizer layout: no master/exp_avg/... keys of ours
    fs_ck = {"model": dict(ck["model"]),
             "last_optimizer_state": {"state": {0: {"step": 11, "exp_avg": torch.zeros(3)}},
                                      "param_groups": [{"lr": 1e-4, "params": [0]}], "loss_scale": 16.0},
             "optimizer_history": [{"criterion_name": "SpeechToUnitMultitaskTaskCriterion",
                                    "optimizer_name": "FP16Optimizer", "num_updates": 11}],
             "extra_state": {"train_iterator": {"epoch": 2, "iterations_in_epoch": 0}}}
    fs_ck["model"]["encoder.layer_norm.weight"] = torch.full_like(fs_ck["model"]["encoder.layer_norm.weight"], 0.5)
    model3 = mm.MMS2UTModel(cfg, device="cpu").init_params(seed=9)
    tr3 = mm.trainer.Trainer(model3, lr=1e-3)
    tr3.opt.exp_avg.fill_(1.0)
    tr3.load_state_dict(fs_ck)
    assert torch.all(model3.params.p["encoder.layer_norm.weight"] == 0.5)
    assert torch.equal(tr3.opt.master, model3.params.flat.float())
    assert torch.all(tr3.opt.exp_avg == 0) and torch.all(tr3.opt.exp_avg_sq == 0)
    assert tr3.completed_updates() == 11 and float(tr3.opt.ost[K.OST_LOSS_SCALE]) == 16.0


def test_layer_arena_layout_queries():
    """The arena / scratch / workspace size queries are consistent with the slots the model reads."""
    K = pkg("kernels")
    lc = K.LayerCall(K._lib.LAYER_DEC, 768, 8, 3072, {}, {}, {})
    lc.a.B, lc.a.T, lc.a.Tk = 4, 151, 125
    nb, offs, mw, sw, _ = lc.sizes()
    rows = 4 * 151
    assert offs[K._lib.SLOT_OUT] + 2 * rows * 768 <= nb and offs[K._lib.SLOT_F1] >= 0 and offs[K._lib.SLOT_XB] >= 0
    assert all(o % 256 == 0 for o in offs if o >= 0)
    assert mw > 0 and sw == 0         # short M: fixups on the main stream; weight gradients grouped, no slabs
    enc = K.LayerCall(K._lib.LAYER_ENC, 768, 8, 3072, {}, {}, {})
    enc.a.B, enc.a.T = 80, 125
    _, eo, emw, esw, _ = enc.sizes()
    assert eo[K._lib.SLOT_XB] == -1 and eo[K._lib.SLOT_Q] == -1 and emw == 0 and esw == 0
