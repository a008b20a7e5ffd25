"""One rank of a world-2 data-parallel run on a single GPU (gloo process group, both ranks
sharing cuda:0) — launched by tests/test_gpu_dp.py as a fresh child process (test infrastructure).

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p MMS2UT_DIST_BACKEND=gloo \
        python tests/dp_child.py OUT_DIR

Runs the real Trainer in its default configuration (deferred chunked Adam, gradient zeroing and
the RCCL/gloo buckets on the low-priority side stream) for 3 updates on this rank's batch, once
per gradient bucket size (0.25 MB: many buckets overlapping the backward; SURVEY §8e's 8 / 25 /
64 / 128 MB), and writes the first update's reduced gradient (taken in stream order right before
the optimizer, Trainer.grad_tap) and the final parameters / optimizer state to
OUT_DIR/rank{r}_b{mb}.npz.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import importlib  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dp_common import BUCKETS_MB, batches, model_cfg  # noqa: E402

mm = importlib.import_module("multimodal-s2ut_amd")


def run(rank, world, bucket_mb, out_dir):
    cfg = model_cfg(mm)
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=5)
    tr = mm.trainer.Trainer(model, lr=1e-3, world_size=world, init_scale=8.0, warmup_updates=0,
                            bucket_mb=bucket_mb)
    assert tr.opt.defer, "the default (deferred Adam) path is the one under test"
    batch = batches(mm, cfg)[rank]
    taps = []
    tr.grad_tap = lambda g: taps.append(g.clone()) if not taps else None
    out = {"nbuckets": np.array(len(tr.reducer.bounds))}
    for step in range(3):
        tr.train_step(batch)
        if step == 0:
            torch.cuda.synchronize()
            out["grad0"] = taps[0].float().cpu().numpy()
            tr.sync()
            out["ost0"] = tr.opt.ost.cpu().numpy()
    tr.sync()
    torch.cuda.synchronize()
    st = tr.opt.stats()
    out["params"] = model.params.flat.cpu().view(torch.int16).numpy()
    out["master"] = tr.opt.master.cpu().numpy()
    out["ost"] = tr.opt.ost.cpu().numpy()
    out["inconsistent"] = np.array(st["inconsistent"])
    np.savez(os.path.join(out_dir, f"rank{rank}_b{bucket_mb:g}.npz"), **out)


def main(out_dir):
    rank, world, local = mm.parallel.init_from_env()
    torch.cuda.set_device(local)
    for mb in BUCKETS_MB:
        run(rank, world, mb, out_dir)
        torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
