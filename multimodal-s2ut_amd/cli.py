"""``mms2ut-train``: the canonical fairseq-train command (scripts/textless/1_train.sh:105-125) on the
HIP path.  Accepts the same flags; data is synthetic Speech-Multi30K-shaped (``--synthetic``), the
TSV/.pth manifest reader being SURVEY §8f's next row.  One process per GPU under
``python -m torch.distributed.run``; batches are dealt round-robin to ranks (fairseq's
ShardedIterator), gradients summed over RCCL (parallel.GradAllReducer).

Log lines follow fairseq's progress format: loss / nll_loss in base 2 per target token, ppl,
wps (target tokens/s), ups, lr, gnorm, loss_scale.
"""
import ast
import json
import math
import sys
import time

import torch

from . import runtime
from .data import SyntheticSpeechMulti30K
from .parallel import init_from_env
from .plugins import REGISTRY, build_parser
from .trainer import Trainer


def main(argv=None):
    args = build_parser().parse_args(argv)
    if not args.fp16:
        raise SystemExit("mms2ut-train: only --fp16 training is implemented (the reference's setting)")
    if args.update_freq != 1:
        raise SystemExit("mms2ut-train: --update-freq 1 only (BASELINE configs)")
    for kind, name in (("task", args.task), ("arch", args.arch), ("criterion", args.criterion)):
        if name not in REGISTRY[kind]:
            raise SystemExit(f"mms2ut-train: unknown {kind} {name!r}; have {sorted(REGISTRY[kind])}")
    if not args.synthetic:
        raise SystemExit("mms2ut-train: manifest (TSV) data loading is not built yet; pass --synthetic")
    rank, world, local = init_from_env()
    dev = torch.device("cuda", local)
    task = REGISTRY["task"][args.task].setup_task(args)
    model = task.build_model(args, device=dev)
    net = model.net
    cfg = net.cfg
    betas = tuple(ast.literal_eval(args.adam_betas))
    tr = Trainer(net, lr=args.lr, betas=betas, clip_norm=args.clip_norm,
                 warmup_updates=args.warmup_updates, warmup_init_lr=args.warmup_init_lr,
                 init_scale=float(args.fp16_init_scale), world_size=world)
    fus = task.multimodal_translation_config
    ds = SyntheticSpeechMulti30K(n_utts=max(64, 2 * args.max_tokens // 400), seed=args.seed,
                                 vocab=cfg["vocab_size"], img_dim=cfg["image_feat_dim"],
                                 with_images=bool(fus is not None and cfg["fusion"]))
    batches = ds.batches(args.max_tokens)
    g = torch.Generator().manual_seed(args.seed)
    upd, t0, ntok = 0, time.time(), 0.0
    while upd < args.max_update:
        order = torch.randperm(len(batches), generator=g).tolist()
        # equal batch count per rank (fairseq pads the last shard with dummy batches)
        order = order[: len(order) // world * world]
        for bi in order[rank::world]:
            sample = ds.sample(batches[bi])
            batch = runtime.prepare_batch(sample, cfg, dev)
            log = tr.train_step(batch)
            ntok += batch.ntokens * world  # rank-local count scaled (no per-step host sync)
            upd += 1
            if upd % args.log_interval == 0 or upd == args.max_update:
                lg = log.tolist()
                st = tr.opt.stats()
                el = time.time() - t0
                if rank == 0:
                    ln2 = math.log(2)
                    rec = {"num_updates": upd, "loss": lg[0] / lg[2] / ln2, "nll_loss": lg[1] / lg[2] / ln2,
                           "ppl": 2 ** (lg[1] / lg[2] / ln2), "wps": ntok / max(el, 1e-9),
                           "ups": upd / max(el, 1e-9), "lr": st["lr"], "gnorm": st["gnorm"],
                           "loss_scale": st["loss_scale"], "overflow": st["overflow"]}
                    print(json.dumps(rec), flush=True)
            if upd >= args.max_update:
                break
    torch.cuda.synchronize(dev)
    return 0


if __name__ == "__main__":
    sys.exit(main())
