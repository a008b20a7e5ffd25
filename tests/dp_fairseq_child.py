"""One rank of a world-2 fairseq drop-in data-parallel run on a single GPU (gloo process group,
both ranks sharing cuda:0) — launched by tests/test_gpu_dp_fairseq.py as a fresh child process
(test infrastructure).

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p MMS2UT_DIST_BACKEND=gloo \
        python tests/dp_fairseq_child.py OUT_DIR TMP_DIR [base]

fairseq-train's distributed path restated (tests/fairseq_stub.py stands in for fairseq, which is
not importable): setup_task -> load_dataset -> build_model -> .half() -> torch DDP with fairseq's
settings (distributed_fairseq_model: bucket_cap_mb 25, broadcast_buffers False,
find_unused_parameters False; a 1 MB variant, and a 25 MB one with find_unused_parameters True
= fairseq --find-unused-parameters) behind fairseq's ModuleProxyWrapper ->
criterion(model, sample) -> loss.backward().  Rank r trains on batch r of the iterator.  Two
iterations per bucket size (DDP rebuilds its buckets in gradient-ready order after the first);
a DDP communication hook logs, per bucket, whether the hand-written backward was still running
when DDP launched it.  Writes OUT_DIR/rank{r}_b{mb}.npz: the averaged gradients of iteration 2
(every parameter, flattened in named_parameters order) and the launch log.
"""
import os
import sys
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import importlib  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import fairseq_stub  # noqa: E402

mm = importlib.import_module("multimodal-s2ut_amd")

NODROP = "--dropout 0 --attention-dropout 0 --relu-dropout 0"
BUCKETS_MB = (25, 1)
RUNS = ((25, False), (1, False), (25, True))   # (bucket MB, find_unused_parameters)
# "base" mode: the base 12 + 6 model (d 768, FFN 3072, 8 heads: 301 MB of fp16 gradients, twelve
# 25 MB buckets), fairseq's default bucket size only
BASE = ("--encoder-layers 12 --decoder-layers 6 --encoder-embed-dim 768 --encoder-ffn-embed-dim 3072 "
        "--encoder-attention-heads 8 --decoder-embed-dim 768 --decoder-ffn-embed-dim 3072 --decoder-attention-heads 8")


class _SetItem:
    """pytest's monkeypatch.setitem for a child process (nothing to undo at exit)."""

    @staticmethod
    def setitem(d, k, v):
        d[k] = v


class ModuleProxyWrapper(torch.nn.Module):
    """fairseq.distributed.ModuleProxyWrapper: forwards attribute access to the DDP-wrapped model
    (criteria call model.get_normalized_probs / model.impl through it)."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module.module, name)

    def forward(self, *a, **k):
        return self.module(*a, **k)


def fusion_yaml():
    from test_gpu_plugins import FUSION_NODROP
    return FUSION_NODROP


def setup(tmp, extra=NODROP):
    os.makedirs(tmp, exist_ok=True)
    fs, regs, args, c, _ = fairseq_stub.dropin_setup(_SetItem(), Path(tmp), fusion_yaml(), extra=extra)
    task = fs.tasks.setup_task(args)
    task.load_dataset("train")
    model = task.build_model(args).half()
    crit = regs["criterion"]["speech_to_unit_v2"].build_criterion(args, task)
    batches = task.get_batch_iterator(task.dataset("train"), max_tokens=450, max_positions=task.max_positions())
    return fs, model, crit, batches


def run(rank, world, bucket_mb, tmp, out_dir, find_unused=False, extra=NODROP):
    tag = f"b{bucket_mb}" + ("u" if find_unused else "")
    fs, model, crit, batches = setup(os.path.join(tmp, f"r{rank}_{tag}"), extra)
    net = model.impl.net
    ddp = torch.nn.parallel.DistributedDataParallel(model, bucket_cap_mb=bucket_mb, broadcast_buffers=False,
                                                    find_unused_parameters=find_unused)
    launches = []

    def hook(state, bucket):
        # parameter groups the hand-written backward has not handed to autograd yet (layers still
        # to be back-propagated) when DDP launches this bucket
        fin = net.grad_release_finish
        rel = fin.__self__ if fin is not None else None
        pending = len(rel.groups) - rel.next if rel is not None else 0
        launches.append((len(launches), pending, bucket.buffer().numel()))
        t = bucket.buffer().div_(world)
        return dist.all_reduce(t, async_op=True).get_future().then(lambda f: f.value()[0])

    ddp.register_comm_hook(None, hook)
    wrapped = ModuleProxyWrapper(ddp)
    model.train()
    sample = fs.utils.apply_half(fs.utils.move_to_cuda(batches[rank]))
    per_iter = []
    for it in range(2):
        model.zero_grad(set_to_none=True)
        launches.clear()
        net.drop.reset(11 + rank)
        loss, ss, log = crit(wrapped, sample)
        loss.backward()
        torch.cuda.synchronize()
        per_iter.append(np.array(launches, dtype=np.int64).reshape(-1, 3))
    g = torch.cat([p.grad.float().flatten() for _, p in model.named_parameters()]).cpu().numpy()
    np.savez(os.path.join(out_dir, f"rank{rank}_{tag}.npz"), grad=g, launches0=per_iter[0],
             launches1=per_iter[1])


def main(out_dir, tmp, mode="tiny"):
    rank, world, local = mm.parallel.init_from_env()
    torch.cuda.set_device(local)
    runs, extra = (((25, False),), NODROP + " " + BASE) if mode == "base" else (RUNS, NODROP)
    for mb, unused in runs:
        run(rank, world, mb, tmp, out_dir, unused, extra)
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(*sys.argv[1:4])
