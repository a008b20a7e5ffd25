"""Host-side (Python) cost of the training step: cProfile over bench.py's workload with the
autograd engine on the calling thread (so the hand-written backward is visible).

usage: python scripts/host_profile.py [--steps 10] [--out gpurun_out/host.prof]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/host.prof")
    a = ap.parse_args()
    torch.autograd.set_multithreading_enabled(False)
    mm = bench.mm
    device = torch.device("cuda", 0)
    cfg = mm.default_cfg()
    model = mm.MMS2UTModel(cfg, device=device).init_params(seed=1)
    tr = bench.trainer_mod.Trainer(model, lr=5e-4, world_size=1)
    fe = bench.frontend_mod.FbankFrontend(device)
    batches = bench.make_batches(cfg, 0, 8, 40000, device, fe)

    def step(i):
        wb, batch = batches[i % len(batches)][:2]
        batch.src = fe(wb)
        tr.train_step(batch)

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    # report any host<->device synchronising torch op issued inside a step
    torch.cuda.set_sync_debug_mode("warn")
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        step(3)
        for x in w[:20]:
            print("SYNC:", str(x.message)[:200], x.filename, x.lineno)
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(a.steps):
        step(3 + i)
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e3 * (t1 - t0) / a.steps:.2f} ms/step (profiled), wall {1e3 * (t2 - t0) / a.steps:.2f}")
    pr.dump_stats(a.out)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(40)
    st.sort_stats("cumtime").print_stats(40)


if __name__ == "__main__":
    main()
