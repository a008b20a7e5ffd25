"""``mms2ut-train``: the canonical fairseq-train command (scripts/textless/1_train.sh:105-125) on the
HIP path.  Accepts the same flags; data is the on-disk manifest (see
below) or synthetic Speech-Multi30K-shaped batches (``--synthetic``).  One process per GPU under
``python -m torch.distributed.run``; batches are dealt round-robin to ranks (fairseq's
ShardedIterator), gradients summed over RCCL (parallel.GradAllReducer).

Log lines follow fairseq's progress format: loss / nll_loss in base 2 per target token, ppl,
wps (target tokens/s), ups, lr, gnorm, loss_scale.

Data: the manifest directory (fairseq's positional DATA: ``{split}.tsv``, ``config.yaml``, WAVs,
image features from the fusion YAML's ``image_feat_path``) through ``manifest.DeviceLoader``, or
``--synthetic``.
"""
import ast
import json
import math
import sys
import time

import torch

from . import data, runtime
from .data import SyntheticSpeechMulti30K
from .parallel import init_from_env
from .plugins import REGISTRY, build_parser
from .trainer import Trainer


def main(argv=None):
    args = build_parser().parse_args(argv)
    if not args.fp16:
        raise SystemExit("mms2ut-train: only --fp16 training is implemented (the reference's setting)")
    if args.update_freq < 1:
        raise SystemExit("mms2ut-train: --update-freq must be >= 1")
    for kind, name in (("task", args.task), ("arch", args.arch), ("criterion", args.criterion)):
        if name not in REGISTRY[kind]:
            raise SystemExit(f"mms2ut-train: unknown {kind} {name!r}; have {sorted(REGISTRY[kind])}")
    if not args.synthetic and not args.data:
        raise SystemExit("mms2ut-train: give the manifest directory (fairseq's DATA argument) or --synthetic")
    rank, world, local = init_from_env()
    dev = torch.device("cuda", local)
    task = REGISTRY["task"][args.task].setup_task(args)
    model = task.build_model(args, device=dev)
    net = model.net
    cfg = net.cfg
    betas = tuple(ast.literal_eval(args.adam_betas))
    tr = Trainer(net, lr=args.lr, betas=betas, clip_norm=args.clip_norm,
                 warmup_updates=args.warmup_updates, warmup_init_lr=args.warmup_init_lr,
                 init_scale=float(args.fp16_init_scale), world_size=world, update_freq=args.update_freq)
    pos = _restore(args, tr, dev)
    fus = task.multimodal_translation_config
    if args.synthetic and cfg.get("multitask"):
        raise SystemExit("mms2ut-train: --multitask-config-yaml needs the on-disk data (text targets per task)")
    if not args.synthetic:
        epoch_updates = _manifest_epochs(args, task, cfg, fus, rank, world, dev)
    else:
        epoch_updates = _synthetic_epochs(args, cfg, fus, rank, world, dev)
    _train_loop(args, tr, rank, world, epoch_updates, pos)
    torch.cuda.synchronize(dev)
    _save(args, tr, rank)
    return 0


def _train_loop(args, tr, rank, world, epoch_updates, pos):
    """fairseq's epoch / update loop.  ``epoch_updates(epoch, skip)`` yields this rank's micro-batch
    lists of one epoch after the first ``skip`` updates (the restored iterator position).  The
    update count is fairseq's num_updates: updates skipped for fp16 overflow do not count.  It is
    read from the device state (identical on every rank) whenever the host's provisional count
    reaches a log / save / stop boundary, so all ranks stop at the same step."""
    upd, epoch, skip = pos["num_updates"], pos["epoch"], pos["iterations_in_epoch"]
    t0, ntok = time.time(), 0.0
    si = args.save_interval_updates
    while upd < args.max_update:
        it = skip
        for micro in epoch_updates(epoch, skip):
            log = tr.train_step(micro)
            ntok += sum(b.ntokens for b in micro) * world  # rank-local count scaled (no per-step host sync)
            it += 1
            upd += 1
            tr.position = {"epoch": epoch, "iterations_in_epoch": it}
            if upd >= args.max_update or upd % args.log_interval == 0 or (si and upd % si == 0):
                upd = tr.completed_updates()
            if upd % args.log_interval == 0 or upd >= args.max_update:
                _log(args, upd, log, tr, ntok, t0, rank)
            if si and upd % si == 0:
                _save(args, tr, rank)
            if upd >= args.max_update:
                return upd
        epoch, skip = epoch + 1, 0
    return upd


def _synthetic_epochs(args, cfg, fus, rank, world, dev):
    # enough utterances that every rank gets at least one update of update_freq micro-batches
    need = max(64, 2 * args.max_tokens // 400) * world * args.update_freq
    ds = SyntheticSpeechMulti30K(n_utts=need, seed=args.seed,
                                 vocab=cfg["vocab_size"], img_dim=cfg["image_feat_dim"],
                                 with_images=bool(fus is not None and cfg["fusion"]))
    batches = ds.batches(args.max_tokens)
    costs = [data.padded_cost([int(ds.lengths[i]) for i in b]) for b in batches]
    uf = args.update_freq

    def epoch_updates(epoch, skip):
        # equal batch count per rank (fairseq pads the last shard with dummy batches); with balanced
        # sharding the ranks of one step get batches of near-equal padded cost
        mine = data.deal_batches(costs, world, args.seed, epoch, balanced=args.balanced_sharding)[rank]
        mine = mine[: len(mine) // uf * uf]
        if not mine:
            raise SystemExit(f"mms2ut-train: {len(batches)} synthetic batches cannot feed {world} ranks x "
                             f"update-freq {uf}")
        for j in range(skip * uf, len(mine), uf):
            yield [runtime.prepare_batch(ds.sample(batches[bi]), cfg, dev) for bi in mine[j:j + uf]]
    return epoch_updates


def _manifest_epochs(args, task, cfg, fus, rank, world, dev):
    """On-disk data: ``{data}/{train_subset}.tsv`` + ``{data}/{config_yaml}``,
    image features from the fusion YAML's ``image_feat_path``; per epoch the length-ordered batches
    are shuffled with (seed, epoch) and dealt to ranks (data.deal_batches)."""
    import os

    from . import data as D
    from . import manifest as M
    if args.target_code_size is None:
        raise SystemExit("mms2ut-train: --target-is-code --target-code-size N is required for unit targets")
    data_cfg = M.load_data_config(os.path.join(args.data, args.config_yaml))
    feat = getattr(fus, "image_feat_path", None) if (fus is not None and cfg["fusion"]) else None
    ds = M.MultiModalS2SManifest(args.data, args.train_subset, M.UnitDictionary.for_codes(args.target_code_size),
                                 data_cfg=data_cfg, image_feat_path=feat,
                                 max_source_positions=cfg.get("max_source_positions", 6000),
                                 max_target_positions=cfg.get("max_target_positions", 1024),
                                 multitask=getattr(task, "multitask_tasks", None))
    uf = args.update_freq

    def epoch_updates(epoch, skip):
        batches = ds.batches(args.max_tokens, seed=args.seed, epoch=epoch, skip_invalid=True)
        costs = [D.padded_cost(ds.n_frames[b].tolist()) for b in batches]
        mine = [batches[i] for i in D.deal_batches(costs, world, args.seed, epoch,
                                                      balanced=args.balanced_sharding)[rank]]
        mine = mine[: len(mine) // uf * uf]
        if not mine:
            raise SystemExit(f"mms2ut-train: {len(batches)} batches cannot feed {world} ranks x update-freq {uf}")
        micro = []
        for batch, _ in M.DeviceLoader(ds, mine[skip * uf:], cfg, dev, seed=args.seed + rank, epoch=epoch):
            micro.append(batch)
            if len(micro) == uf:
                yield micro
                micro = []
    return epoch_updates


def _save(args, tr, rank):
    """--save-dir: fairseq-layout checkpoint_last.pt — model (MM_S2UTTransformerModel keys),
    last_optimizer_state (fp32 master / Adam moments / device state, loss_scale), optimizer_history,
    extra_state (num_updates, train_iterator position), args (argparse.Namespace) — written by rank 0
    (fairseq checkpoint_utils.save_checkpoint)."""
    import argparse
    import os
    if not args.save_dir:
        return
    # a run that went FATAL (sticky) since the last log boundary raises here, on every rank, instead
    # of writing a checkpoint that could never apply another update (fairseq raises at the step)
    tr.opt.check_fatal()
    state = tr.state_dict()          # every rank syncs; only rank 0 writes
    if rank != 0:
        return
    os.makedirs(args.save_dir, exist_ok=True)
    state["args"] = argparse.Namespace(**{k: v for k, v in vars(args).items()
                                          if isinstance(v, (int, float, str, bool, type(None)))})
    path = os.path.join(args.save_dir, "checkpoint_last.pt")
    torch.save(state, path + ".tmp")
    os.replace(path + ".tmp", path)


def _restore(args, tr, dev):
    """--restore-file (default checkpoint_last.pt in --save-dir, as fairseq) -> the iterator
    position {num_updates, epoch, iterations_in_epoch} to resume from.  The file is read with
    ``weights_only=True`` (argparse.Namespace allow-listed for the ``args`` entry)."""
    import argparse
    import os
    pos = {"num_updates": 0, "epoch": 1, "iterations_in_epoch": 0}
    path = args.restore_file
    if path and not os.path.isabs(path) and args.save_dir:
        path = os.path.join(args.save_dir, path)
    if not path or not os.path.exists(path):
        if args.restore_file and args.restore_file != "checkpoint_last.pt":
            raise SystemExit(f"mms2ut-train: --restore-file {args.restore_file} not found")
        return pos
    with torch.serialization.safe_globals([argparse.Namespace]):
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
    tr.load_state_dict(ckpt)
    es = ckpt.get("extra_state") or {}
    ti = es.get("train_iterator") or {}
    pos.update(num_updates=tr.completed_updates(), epoch=int(ti.get("epoch", 1)),
               iterations_in_epoch=int(ti.get("iterations_in_epoch", 0)))
    # a resume that is already at --max-update saves this position again, not the default one
    tr.position = {"epoch": pos["epoch"], "iterations_in_epoch": pos["iterations_in_epoch"]}
    return pos


def _log(args, upd, log, tr, ntok, t0, rank):
    """Every rank reads the (identical) device optimizer state at the log cadence and raises on a
    sticky FATAL state together (FP16Adam.check_fatal); rank 0 prints the record."""
    st = tr.opt.check_fatal()
    if rank != 0:
        return
    lg = log.tolist()
    el = time.time() - t0
    ln2 = math.log(2)
    rec = {"num_updates": upd, "loss": lg[0] / lg[2] / ln2, "nll_loss": lg[1] / lg[2] / ln2,
           "ppl": 2 ** (lg[1] / lg[2] / ln2), "wps": ntok / max(el, 1e-9), "ups": upd / max(el, 1e-9),
           "lr": st["lr"], "gnorm": st["gnorm"], "loss_scale": st["loss_scale"], "overflow": st["overflow"]}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    sys.exit(main())
