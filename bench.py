"""Benchmark: mm_s2ut_transformer fp16 training throughput (audio frames / s / node).

One step = one full training update on one max-tokens-40000 batch per rank: GPU fbank front end
(waveforms already resident in HBM) -> Conv1d subsampler -> 12-layer encoder -> gated image fusion
-> 6-layer unit decoder -> label-smoothed CE -> hand-written backward with bucketed RCCL all-reduce
-> FP16Optimizer/Adam.  Synthetic Speech-Multi30K-shaped data, random-init weights.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints ONE JSON line (value = frames processed by all ranks / max-over-ranks wall time).
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
mm = importlib.import_module("multimodal-s2ut_amd")
from importlib import import_module  # noqa: E402

data = import_module("multimodal-s2ut_amd.data")
frontend_mod = import_module("multimodal-s2ut_amd.frontend")
runtime = import_module("multimodal-s2ut_amd.runtime")
kernels = import_module("multimodal-s2ut_amd.kernels")
parallel = import_module("multimodal-s2ut_amd.parallel")
trainer_mod = import_module("multimodal-s2ut_amd.trainer")
model_mod = import_module("multimodal-s2ut_amd.model")

MFMA_PEAK_F16 = 2500.0   # TFLOP/s dense fp16 (MI355X_MICROARCH.md chip parameters)
HBM_PEAK = 8000.0        # GB/s spec


def fwd_flops_per_utt(Ts, Tt, cfg, Ti=577, Di=768, fusion=True, split=False):
    """SURVEY.md §8(d) closed form (true lengths), forward FLOPs of one utterance.
    split=True -> (total, multi-head attention score/PV FLOPs run by the fused attention kernel)."""
    d, F, C, V = cfg["encoder_embed_dim"], cfg["encoder_ffn_embed_dim"], cfg["conv_channels"], cfg["vocab_size"]
    T1 = (Ts - 1) // 2 + 1
    Te = (T1 - 1) // 2 + 1
    f = 2 * T1 * (80 * 5 * C) + 2 * Te * (C // 2 * 5 * 2 * d)
    f += cfg["encoder_layers"] * (Te * (8 * d * d + 4 * d * F) + 4 * Te * Te * d)
    if fusion:
        k = 1 if cfg["multimodal_attention_type"] == "multimodal_attention" else 0
        f += Te * 8 * d * d + 4 * Ti * Di * d + 4 * Te * (Ti + k) * d
    f += cfg["decoder_layers"] * (Tt * (12 * d * d + 4 * d * F) + 4 * Tt * Tt * d + 4 * Te * d * d + 4 * Tt * Te * d)
    f += 2 * Tt * d * V
    mha = cfg["encoder_layers"] * 4 * Te * Te * d + cfg["decoder_layers"] * (4 * Tt * Tt * d + 4 * Tt * Te * d)
    return (f, mha) if split else f


def make_batches(cfg, rank, nb, max_tokens, device, frontend, n_utts=3000, img_tokens=577):
    """nb length-bucketed batches (fairseq batch_by_size), spread evenly over the length
    distribution of a synthetic corpus; everything moved to HBM before timing."""
    corpus = data.SyntheticSpeechMulti30K(n_utts=n_utts, seed=1 + rank, img_tokens=img_tokens,
                                          img_dim=cfg["image_feat_dim"], with_images=cfg["fusion"])
    all_b = corpus.batches(max_tokens)
    pick = [all_b[int(i)] for i in np.linspace(0, len(all_b) - 1, nb).round()]
    out = []
    for bi, idx in enumerate(pick):
        items = [corpus.item(i, features=False) for i in idx]
        rng = np.random.default_rng((rank, bi))
        waves = []
        for it in items:
            n = 160 * it["n_frames"] + 240
            t = np.arange(n) / 16000.0
            w = (0.1 * rng.standard_normal(n) + 0.3 * np.sin(2 * np.pi * 440.0 * t)) * 2 ** 15
            waves.append(w.astype(np.float32))
            it["source"] = torch.zeros(it["n_frames"], 80)  # placeholder: features come from the GPU fbank
        wb = frontend.upload(waves)
        sample = data.collater(items)
        assert sample["net_input"]["src_lengths"].tolist() == wb["n_frames"].tolist()
        sample["net_input"]["src_tokens"] = None
        src_dummy = torch.empty(wb["B"], wb["Tmax"], 80, dtype=torch.float16, device=device)
        batch = runtime.prepare_batch(sample, cfg, device, src_override=src_dummy)
        tl = sample["target_lengths"].numpy()
        sl = sample["net_input"]["src_lengths"].numpy()
        parts = [fwd_flops_per_utt(int(s), int(t), cfg, Ti=img_tokens, Di=cfg["image_feat_dim"], fusion=cfg["fusion"],
                                   split=True) for s, t in zip(sl, tl)]
        flops = sum(p[0] for p in parts)
        mha = sum(p[1] for p in parts)
        # GEMM-kernel share of the algorithmic FLOPs: everything but the multi-head attention
        # products, which the fused attention kernel executes (the fusion attention stays on GEMMs)
        gemm_flops = flops - mha
        # host copies of the first batch's waveforms (collated order) for the CPU baseline's fbank
        host_waves = [waves[i] for i in wb["order"]] if bi == 0 else None
        out.append((wb, batch, sample, 3 * flops, 3 * gemm_flops, host_waves))
    return out


def gemm_pmc_traffic():
    """Measured HBM bytes per GEMM launch: the newest profiles/*_gemm_traffic.json, written by
    scripts/pmc_traffic.py from separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes over this bench
    (gfx950 FETCH x2 correction).  A PMC pass cannot run inside the timed bench itself."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_gemm_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("gemm_hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo) for the cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cycle_batches(steps, nbatches):
    """Resident batch count for a K-step timed window: the largest divisor of K that is <= the
    requested count, so the window is whole cycles of the resident set and the batch mix (hence
    frames/s) does not depend on --steps beyond that choice."""
    return max(d for d in range(1, max(1, min(steps, nbatches)) + 1) if steps % d == 0)


def cpu_baseline(cfg, model, sample, waves, budget_s=20.0, target_frames=3000):
    """The oracle (fp32 PyTorch-CPU restatement) timed on the host cores on a bounded sample of the
    same workload, like for like with the GPU step: the first utterances of
    the bench's first batch (the GPU's own waveforms, image features and targets, up to
    ``target_frames`` source frames), per step the Kaldi fbank + utterance CMVN of their waveforms
    (oracle/ref_fbank.py), collation, the model forward with every dropout site on (Bernoulli
    masks drawn on the CPU), backward and the FP16Optimizer/Adam update."""
    from oracle import ref_fbank as RF
    from oracle import ref_model as R
    ocfg = dict(cfg)
    sd = {k: v.detach().float().cpu() for k, v in model.params.p.items()}
    P = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ni = sample["net_input"]
    lens = ni["src_lengths"].tolist()
    n = 1
    while n < len(lens) and sum(lens[:n + 1]) <= target_frames:
        n += 1
    frames = int(sum(lens[:n]))
    tt = int((sample["target"][:n] != 1).sum(1).max())
    drop = R.CPUDropout(seed=1)
    states = {k: (torch.zeros_like(v), torch.zeros_like(v)) for k, v in P.items()}
    masters = {k: v.detach().clone() for k, v in P.items()}

    def step(i):
        feats = [RF.utterance_cmvn(RF.fbank(w)) for w in waves[:n]]
        src = torch.zeros(n, max(f.shape[0] for f in feats), 80)
        for b, f in enumerate(feats):
            src[b, :f.shape[0]] = torch.from_numpy(f)
        sub = {"net_input": {"src_tokens": src, "src_lengths": ni["src_lengths"][:n].clone(),
                             "prev_output_tokens": ni["prev_output_tokens"][:n, :tt],
                             "imgs_list": [ni["imgs_list"][0][:n].float()] if ni["imgs_list"] else [],
                             "img_masks_list": [None] if ni["imgs_list"] else []},
               "target": sample["target"][:n, :tt]}
        for v in P.values():
            v.grad = None
        loss, _, _ = R.model_forward(P, sub, ocfg, masks=drop)
        loss.backward()
        names = list(P)
        R.fp16_optimizer_step([masters[k] for k in names], [P[k].grad.half() for k in names],
                              [states[k] for k in names], i + 1, 1e-4, 1.0 / frames)

    step(0)
    t0 = time.time()
    k = 0
    while True:
        step(k + 1)
        k += 1
        if time.time() - t0 > budget_s or k >= 20:
            break
    dt = time.time() - t0
    return {"value": frames * k / dt, "unit": "audio-frames/s", "cores": torch.get_num_threads(),
            "cpu": cpu_model(), "kind": "port",
            "sample": f"oracle fp32 training step on the first B={n} utterances ({frames} source frames, "
                      f"{tt} target positions) of the bench's first batch: Kaldi fbank + utterance CMVN of their "
                      f"waveforms, forward with dropout on at every site (CPU-drawn masks), backward, "
                      f"FP16Optimizer/Adam; {k} steps in {dt:.1f}s on {torch.get_num_threads()} threads"}


def decode_cpu_baseline(model, sample, beam, budget_s=20.0):
    """The oracle's beam search (oracle/ref_generate.py over the fp32 oracle decoder re-run per
    prefix — the reference has no incremental CPU path here) on a bounded sample: one utterance,
    the bench's beam, as many steps as fit the budget (each step re-decodes every prefix)."""
    from oracle import ref_generate as RG
    from oracle import ref_model as R
    cfg = R.no_dropout(dict(model.cfg))
    P = {k: v.detach().float().cpu() for k, v in model.params.p.items()}
    ni = sample["net_input"]
    with torch.no_grad():
        enc, pad, _ = R.encoder_forward(P, ni["src_tokens"][:1].float(), ni["src_lengths"][:1], cfg,
                                        imgs=ni["imgs_list"][0][:1].float() if ni["imgs_list"] else None)
    step_fn = RG.full_recompute_step(P, cfg, enc, pad, beam)
    t0 = time.time()
    steps = 0
    for T in range(4, 64, 4):
        RG.beam_search(step_fn, 1, cfg["vocab_size"], beam, T, min_len=T + 1)   # forced to run T steps
        steps += T + 1
        if time.time() - t0 > budget_s:
            break
    dt = time.time() - t0
    return {"value": steps * beam / dt, "unit": "hypothesis-tokens/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle beam search (fp32 decoder re-run over every prefix), 1 utterance, beam {beam}, "
                      f"{steps} decoder steps in {dt:.1f}s"}


def decode_main(args):
    """--decode: beam-search inference (fairseq-generate --beam 10 --max-len-a 1)
    on the base model: one JSON line of hypothesis-tokens/s with the decode self-attention roofline
    and the oracle CPU baseline.  Random weights rarely emit </s>: every hypothesis decodes to
    max_len (the longest decode)."""
    gen_mod = import_module("multimodal-s2ut_amd.generate")
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    cfg = mm.default_cfg()
    model = mm.MMS2UTModel(cfg, device=device).init_params(seed=1)
    bsz, frames, beam = args.decode_bsz, args.decode_frames, 10
    sample = data.make_sample([frames] * bsz, [10] * bsz, img_tokens=577, img_dim=768, seed=0)
    batch = runtime.prepare_batch(sample, model.cfg, device)
    gen_mod.generate(model, batch, beam_size=beam, max_len_a=1.0, max_len_b=200)   # warmup + graph capture
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hyps = gen_mod.generate(model, batch, beam_size=beam, max_len_a=1.0, max_len_b=200)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = max(len(h["tokens"]) for hs in hyps for h in hs)
    N, H, hd = bsz * beam, cfg["decoder_attention_heads"], cfg["decoder_embed_dim"] // cfg["decoder_attention_heads"]
    # decode self-attention: every cached K and V row of every hypothesis read once per layer-step
    attn_bytes = sum(N * H * t * hd * 2 * 2 for t in range(1, steps + 1)) * cfg["decoder_layers"]
    cpu = None if args.no_cpu_baseline else decode_cpu_baseline(model, sample, beam, args.cpu_budget)
    print(json.dumps({
        "metric": "beam-search decode hypothesis-tokens/s (fairseq-generate --beam 10 --max-len-a 1)",
        "value": steps * N / dt, "unit": "hypothesis-tokens/s", "n_gpus": 1, "steps": steps,
        "ms_per_step": 1e3 * dt / steps, "higher_is_better": True, "vs_baseline": None, "dtype": "fp16",
        "data": "synthetic (random-init weights: every hypothesis runs to max_len)",
        "config": {"workload": f"mm_s2ut_transformer base, {bsz} x {frames}-frame utterances, beam {beam}",
                   "sentences_per_s": bsz / dt},
        "roofline": {"bound": "hbm", "kernel": "decode_attn_kernel (self-attention over the KV cache)",
                     "algorithmic_bytes_per_step": attn_bytes / steps, "peak": HBM_PEAK, "unit": "GB/s",
                     "note": "achieved GB/s of this kernel comes from its rocprof duration: "
                             "profiles/round1_v6_generate_kernel_stats.csv (4.0 TB/s measured)"},
        "cpu_baseline": cpu}), flush=True)


def launch_ranks(args):
    """``--gpus N`` without a torch.distributed launcher around us: start ``torch.distributed.run
    --nproc-per-node N`` over this same script as a CHILD process (this process has not touched the
    GPU: nothing above this point initialises HIP) and exit with its return code; rank 0's JSON line
    reaches stdout through the inherited file descriptors.  Under a launcher (WORLD_SIZE set), the
    launcher's world size must equal --gpus: a mismatch fails loudly instead of timing a different
    node size than the one asked for.  Returns only when this process is itself a rank."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
        return
    if args.gpus <= 1:
        return
    import socket
    import subprocess
    backend = os.environ.get("MMS2UT_DIST_BACKEND", "")
    ndev = torch.cuda.device_count()       # does not initialise the GPU on this image
    if backend != "gloo" and ndev < args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but {ndev} visible GPUs (RCCL needs one GPU per rank; "
                         f"MMS2UT_DIST_BACKEND=gloo rehearses N ranks on fewer devices)")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = subprocess.call(cmd, env=env)
    sys.exit(rc)


def host_issue_cost(step, base, n, world):
    """ms of host CPU (main thread + the autograd thread running the hand-written backward) to
    enqueue one training step, measured one step at a time: the device is idle when each step
    starts, so no launch waits for queue space; the synchronize between steps is outside the
    measured interval."""
    cpu = 0.0
    for i in range(n):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        c0, b0 = time.thread_time(), runtime.BWD_CPU_S[0]
        step(base + i)
        cpu += time.thread_time() - c0 + runtime.BWD_CPU_S[0] - b0
    torch.cuda.synchronize()
    return 1e3 * cpu / max(n, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--max-tokens", type=int, default=40000)
    ap.add_argument("--nbatches", type=int, default=8)
    ap.add_argument("--audio-only", action="store_true", help="BASELINE configs[3]: no fusion tail")
    ap.add_argument("--image-feats", choices=("vit", "detr"), default="vit",
                    help="detr = BASELINE configs[4]: DETR feats [100, 256], SA_image_dropout 0.5, "
                         "modality_dropout = audio_dropout = 0.5")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--graph", choices=("on", "off"), default="off",
                    help="replay each training step as a captured HIP graph (world size 1).  Off by "
                         "default: ROCm 7 executes the captured step without the weight-gradient "
                         "side stream's overlap (22.6 ms vs 18.3 ms eager, DESIGN.md §7)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gemm-timing", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--decode", action="store_true", help="beam-search inference line instead of training")
    ap.add_argument("--decode-bsz", type=int, default=16)
    ap.add_argument("--decode-frames", type=int, default=300)
    args = ap.parse_args()
    if args.decode:
        return decode_main(args)
    launch_ranks(args)

    rank, world, local = parallel.init_from_env()
    if world > 1:
        world = dist.get_world_size()          # n_gpus as the process group sees it
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    detr = args.image_feats == "detr"
    img_tokens = 100 if detr else 577
    cfg = mm.default_cfg(fusion=not args.audio_only, **(dict(image_feat_dim=256, SA_image_dropout=0.5,
                                                             modality_dropout=0.5, audio_dropout=0.5)
                                                        if detr else {}))
    model = mm.MMS2UTModel(cfg, device=device).init_params(seed=1)
    graph = args.graph == "on"
    tr = trainer_mod.Trainer(model, lr=5e-4, world_size=world, bucket_mb=args.bucket_mb, graph=graph)
    fe = frontend_mod.FbankFrontend(device)
    nb = cycle_batches(args.steps, args.nbatches)
    batches = make_batches(cfg, rank, nb, args.max_tokens, device, fe, img_tokens=img_tokens)

    def step(i, eager=False, draws=None):
        wb, batch = batches[i % len(batches)][:2]

        def frontend():     # GPU fbank + CMVN of the resident waveforms, part of the step
            batch.src = fe(wb)
        tr.train_step(batch, prologue=frontend, eager=eager, draws=draws)

    # untimed loss-scale settling: the fp16 optimizer starts at scale 128 (fairseq --fp16-init-scale)
    # and skips the update of every overflowing step while it halves the scale; run until a step
    # completes (the overflow flag is the all-reduced one, identical on every rank) so the timed
    # steps are complete optimizer steps
    settle = 0
    while settle < 16:
        step(settle)
        settle += 1
        if not tr.opt.stats()["overflow"]:
            break
    for i in range(args.warmup):
        step(i)
    n_graphs = 0
    if graph:
        # capture every (batch, modality-dropout branch) the timed window can meet, so no capture
        # lands inside it (each first encounter is one eager update + a capture; replays follow)
        branches = [(0.99, 0.99)]
        if cfg["modality_dropout"] > 0:
            if cfg["audio_dropout"] > 0:
                branches.append((0.0, 0.0))
            if cfg["audio_dropout"] < 1:
                branches.append((0.0, 0.99))
        for i in range(len(batches)):
            for dr in branches:
                step(i, draws=[dr])
        n_graphs = len(tr.graphs)
    base = args.warmup   # the timed batch sequence does not depend on how many settling steps ran
    host_cpu = [0.0]   # CPU seconds of the issuing threads (main + autograd backward) in the last window

    def timed(profile):
        """K steps between barrier + synchronize on both sides -> (seconds, host issue seconds, GEMM stats).
        profile=True: the roofline pass — every GEMM kernel's workgroups store their start / end
        s_memrealtime ticks (mms2ut_profile_stamps), with the weight-gradient side stream folded
        into the main stream so no two GEMMs overlap: a launch's duration is max(end) - min(start)
        over its workgroups, the dispatch span rocprofv3 reports, without the 1.3-1.5x inflation
        per-launch HIP event pairs added to 20-90 us kernels (round 2 measurement)."""
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        side_was = kernels._Side.enabled
        stamps = None
        if profile:
            kernels._Side.enabled = False
            kernels.gemm_profile_begin(2000 * args.steps)
            # in-kernel block stamps (2 x int64 per workgroup; ~0.2 M workgroups per step)
            stamps = torch.zeros(2 * 400_000 * args.steps, dtype=torch.int64, device=device)
            kernels.gemm_profile_stamps(stamps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        prof = bprof = None
        if not profile and os.environ.get("MMS2UT_HOST_PROFILE"):
            import cProfile
            prof = cProfile.Profile()
            bprof = cProfile.Profile()
            runtime._BWD_PROFILE = bprof
            prof.enable()
        c0, b0 = time.thread_time(), runtime.BWD_CPU_S[0]
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(base + i, eager=profile)
        t_issue = time.perf_counter()  # host finished enqueueing (host-bound if ~ t1)
        host_cpu[0] = time.thread_time() - c0 + runtime.BWD_CPU_S[0] - b0
        if prof is not None:
            import pstats
            prof.disable()
            runtime._BWD_PROFILE = None
            print("== host profile: main thread (forward, loss, optimizer)", file=sys.stderr)
            pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(30)
            print("== host profile: autograd thread (hand-written backward)", file=sys.stderr)
            pstats.Stats(bprof, stream=sys.stderr).sort_stats("tottime").print_stats(30)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        g = (0.0, 0, 0.0, 0.0)
        launches = None
        if profile:
            g = kernels.gemm_profile_end()
            _, l_fl, l_cls = kernels.gemm_profile_launches(g[1])
            l_ms = kernels.gemm_profile_durations(stamps, g[1])
            if np.isnan(l_ms).any():
                raise SystemExit(f"bench: GEMM stamp buffer overflowed ({int(np.isnan(l_ms).sum())} launches)")
            launches = (l_ms, l_fl, l_cls)
            g = (float(l_ms.sum()), g[1], g[2], g[3])
            kernels._Side.enabled = side_was
        return t1 - t0, t_issue - t0, g, launches

    # the throughput region runs uninstrumented; the same K steps are then re-run serially with the
    # library's in-kernel workgroup stamps for the roofline
    t_run, t_issue_run, _, _ = timed(False)
    host_cpu_run = host_cpu[0]
    host_cost = host_issue_cost(step, base, min(args.steps, 5), world)
    t_prof = None
    gemm_ms, n_launch, launched_flops, gemm_bytes = 0.0, 0, 0.0, 0.0
    classes, templates = {}, {}
    if not args.no_gemm_timing:
        t_prof, _, (gemm_ms, n_launch, launched_flops, gemm_bytes), (l_ms, l_fl, l_cls) = timed(True)
        if os.environ.get("MMS2UT_GEMM_DUMP"):
            # per-launch table of the roofline pass (scripts/gemm_table.py summarises it)
            np.savez(os.environ["MMS2UT_GEMM_DUMP"], ms=l_ms, flops=l_fl, cls=l_cls,
                     mnk=kernels.gemm_profile_shapes(int(n_launch)), steps=args.steps)
        for ms_, fl_, c_ in zip(l_ms.tolist(), l_fl.tolist(), l_cls.tolist()):
            if c_ & 256:
                name = "batched (fusion attention QK^T / PV)"
            elif not (c_ & 1) and not (c_ & 2):
                name = "weight gradient (TN: grouped unsplit, or split-K slabs)"
            else:
                name = "forward / dgrad (NT, fused epilogues)"
            e = classes.setdefault(name, [0.0, 0.0, 0])
            e[0] += ms_
            e[1] += fl_
            e[2] += 1
            # per kernel template (rocprofv3 names them gemm_dma_kernel<A_KC, B_KC, EPI, ...>)
            t = f"gemm<{'true' if c_ & 1 else 'false'}, {'true' if c_ & 2 else 'false'}, {(c_ >> 2) & 63}>" + \
                (" batched" if c_ & 256 else "") + (" split-K" if c_ & 512 else "") + (" grouped" if c_ & 1024 else "") + \
                (" short-M" if c_ & 2048 else "")
            e = templates.setdefault(t, [0.0, 0.0, 0])
            e[0] += ms_
            e[1] += fl_
            e[2] += 1
    t0, t1, t_issue = 0.0, t_run, t_issue_run
    elapsed = t1 - t0
    frames = sum(int(batches[(base + i) % len(batches)][1].n_src_frames) for i in range(args.steps))
    alg_flops = sum(batches[(base + i) % len(batches)][4] for i in range(args.steps))
    total_flops = sum(batches[(base + i) % len(batches)][3] for i in range(args.steps))
    stats = torch.tensor([elapsed, frames, alg_flops, gemm_ms, n_launch, total_flops], dtype=torch.float64,
                         device=device)
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        frames_all = float(sm[1])
        flops_all, gemm_all, nl_all, total_flops_all = float(sm[2]), float(sm[3]), float(sm[4]), float(sm[5])
    else:
        frames_all, flops_all, gemm_all, nl_all = float(frames), float(alg_flops), gemm_ms, float(n_launch)
        total_flops_all = float(total_flops)
    ost = dict(tr.opt.stats(), untimed_scale_settling_steps=settle)
    # fp32 master checksum after every step above: equal on all ranks (DP keeps replicas identical)
    # and, for a fixed step sequence, independent of --bucket-mb (scripts/_dp2_rehearsal.sh)
    tr.sync()
    ck = torch.tensor([float(tr.opt.master.double().sum())], dtype=torch.float64, device=device)
    ost["master_checksum"] = float(ck)
    if world > 1:
        cks = [torch.zeros_like(ck) for _ in range(world)]
        dist.all_gather(cks, ck)
        ost["ranks_identical"] = all(float(c) == float(ck) for c in cks)
    traffic, traffic_src = gemm_pmc_traffic()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, model, batches[0][2], batches[0][5], args.cpu_budget)
    if rank == 0:
        achieved = (flops_all / (gemm_all / 1e3) / 1e12) if gemm_all > 0 else None
        class_lines = {k: {"ms_per_step": v[0] / args.steps, "launches_per_step": v[2] / args.steps,
                           "launched_tflops": v[1] / max(v[0], 1e-9) / 1e9,
                           "frac": v[1] / max(v[0], 1e-9) / 1e9 / MFMA_PEAK_F16}
                       for k, v in classes.items()}
        dominant = None
        if class_lines:
            dn = max(class_lines, key=lambda k: class_lines[k]["ms_per_step"])
            dominant = dict(class_lines[dn], name=dn)
        tmpl_lines = {k: {"us_per_launch": 1e3 * v[0] / max(v[2], 1), "launches_per_step": v[2] / args.steps,
                          "ms_per_step": v[0] / args.steps, "launched_tflops": v[1] / max(v[0], 1e-9) / 1e9,
                          "frac": v[1] / max(v[0], 1e-9) / 1e9 / MFMA_PEAK_F16}
                      for k, v in sorted(templates.items(), key=lambda kv: -kv[1][0])}
        line = {
            "metric": "audio-frames/sec/node, mm_s2ut_transformer fp16, max-tokens 40000, 1/2/4/8 GPUs",
            "value": frames_all / elapsed,
            "unit": "audio-frames/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp16", "data": "synthetic (Speech-Multi30K-shaped; random-init weights)",
            "config": {"workload": ("mm_s2ut_transformer base audio-only" if args.audio_only else
                                    "mm_s2ut_transformer base (DETR-256 x 100 image feats, SA_image_dropout 0.5, "
                                    "modality/audio dropout 0.5)" if detr else
                                    "mm_s2ut_transformer base (ViT-768 image feats, multimodal_attention+gate)"),
                       "model": "mm_s2ut_transformer", "max_tokens": args.max_tokens,
                       "global_batch_frames_per_step": frames_all / args.steps,
                       "parallelism": f"dp{world}", "front_end": "GPU fbank+CMVN in step",
                       "alg_flops_per_frame": total_flops_all / max(frames_all, 1),
                       "model_tflops_per_s": total_flops_all / elapsed / 1e12},
            "roofline": {"bound": "mfma", "kernel": "mms2ut GEMM family (gemm_dma / gemm256p, all launches)",
                         "achieved": achieved, "peak": MFMA_PEAK_F16, "unit": "TFLOP/s",
                         "frac": (achieved / MFMA_PEAK_F16) if achieved else None, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": gemm_bytes / max(n_launch, 1),
                         "gemm_ms_per_step": gemm_all / world / args.steps,
                         "gemm_launches_per_step": nl_all / world / args.steps,
                         "gemm_launched_tflops": launched_flops / max(gemm_ms, 1e-9) / 1e9,
                         "dominant": dominant,
                         "classes": class_lines,
                         "kernels": tmpl_lines,
                         "host_issue_ms_per_step": 1e3 * (t_issue - t0) / args.steps,
                         # CPU time of the two issuing threads (main: forward, loss, optimizer;
                         # autograd's: the hand-written backward) — the host's own cost per step,
                         # without the waits on the runtime the wall-clock issue time includes
                         # the host's own issue cost: one step at a time (synchronised after each,
                         # outside the measured interval), so the HIP runtime's run-ahead throttle —
                         # a busy wait once a queue is full, counted as CPU time by the overlapped
                         # window — does not enter; the overlapped window's figure beside it
                         "host_cpu_ms_per_step": host_cost,
                         "host_cpu_ms_per_step_overlapped": 1e3 * host_cpu_run / args.steps,
                         "hip_graph": {"enabled": graph, "graphs": n_graphs},
                         "roofline_pass_ms_per_step": (1e3 * t_prof / args.steps) if t_prof else None,
                         "note": "achieved = SURVEY §8d algorithmic GEMM FLOPs (true lengths, 3x fwd, "
                                 "multi-head attention products excluded) / summed kernel durations of every "
                                 "GEMM launch, measured on a second pass of the same K steps run serially "
                                 "(side stream folded into the main one): each workgroup stores its "
                                 "s_memrealtime start / end ticks, a launch lasts max(end) - min(start) over "
                                 "its workgroups (split-K fixup included); value comes from the "
                                 "uninstrumented overlapped pass. classes/dominant/kernels: launched "
                                 "(padded-shape) FLOPs / kernel time; kernels are keyed like rocprofv3's "
                                 "gemm_dma_kernel<A_KC, B_KC, EPI, ...> names"},
            "cpu_baseline": cpu,
            "optimizer": ost,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
