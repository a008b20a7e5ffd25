"""One rank of a world-2 data-parallel run on a single GPU (gloo process group, both ranks
sharing cuda:0) — launched by tests/test_gpu_dp.py as a fresh child process (test infrastructure).

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p MMS2UT_DIST_BACKEND=gloo \
        python tests/dp_child.py OUT_DIR

Runs the real Trainer (bucketed reducer with DDP pre-division, grad-norm consistency check)
for 3 updates on this rank's batch and writes the first update's reduced gradient and the final
parameters / optimizer state to OUT_DIR/rank{r}.npz.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import importlib  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dp_common import batches, model_cfg  # noqa: E402

mm = importlib.import_module("multimodal-s2ut_amd")


def main(out_dir):
    rank, world, local = mm.parallel.init_from_env()
    torch.cuda.set_device(local)
    cfg = model_cfg(mm)
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=5)
    tr = mm.trainer.Trainer(model, lr=1e-3, world_size=world, init_scale=8.0, warmup_updates=0,
                            bucket_mb=0.25)          # many buckets: exercises the overlap path
    batch = batches(mm, cfg)[rank]
    out = {}
    for step in range(3):
        tr.train_step(batch)
        torch.cuda.synchronize()
        if step == 0:
            out["grad0"] = model.params.grad.float().cpu().numpy()
            out["ost0"] = tr.opt.ost.cpu().numpy()
    tr.sync()
    torch.cuda.synchronize()
    st = tr.opt.stats()
    out["params"] = model.params.flat.cpu().view(torch.int16).numpy()
    out["master"] = tr.opt.master.cpu().numpy()
    out["ost"] = tr.opt.ost.cpu().numpy()
    out["inconsistent"] = np.array(st["inconsistent"])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
