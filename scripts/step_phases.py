"""Wall time of the training step's phases on the main (trainer) stream, with the weight-gradient
side stream overlapping as in bench.py: front end + forward + loss | backward (ends at the side
join) | optimizer.  HIP events on the trainer's stream; bench batches and settings.

    python scripts/step_phases.py [steps]
"""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = importlib.import_module("bench")
mm = bench.mm
runtime, trainer_mod, kernels = bench.runtime, bench.trainer_mod, bench.kernels


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    cfg = mm.default_cfg()
    model = mm.MMS2UTModel(cfg, device=device).init_params(seed=1)
    tr = trainer_mod.Trainer(model, lr=5e-4, world_size=1)
    fe = bench.frontend_mod.FbankFrontend(device)
    nb = bench.cycle_batches(steps, 8)
    batches = bench.make_batches(cfg, 0, nb, 40000, device, fe)
    m = model

    def one(i, ev):
        wb, batch = batches[i % len(batches)][:2]
        with torch.cuda.stream(tr.stream):
            ev[0].record()
            batch.src = fe(wb)
            logits, aux = runtime.model_outputs(m, [batch][0])
            m.params.await_all()
            if m.params.zero_each_step:
                m.params.grad.zero_()
            loss, nll = runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"], cfg["label_smoothing"],
                                                  cfg["padding_idx"])
            del logits
            ev[1].record()
            loss.backward(tr.opt.loss_scale())
            ev[2].record()
            tr.log[trainer_mod.LOG_SS_OVER_WORLD].fill_(float(batch.ntokens))
            tr.opt.step(tr.log[trainer_mod.LOG_SS_OVER_WORLD:trainer_mod.LOG_SS_OVER_WORLD + 1])
            ev[3].record()

    for i in range(8):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        one(i, ev)
    torch.cuda.synchronize()
    acc = [0.0, 0.0, 0.0]
    evs = []
    for i in range(steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        one(i, ev)
        evs.append(ev)
    torch.cuda.synchronize()
    for ev in evs:
        for k in range(3):
            acc[k] += ev[k].elapsed_time(ev[k + 1])
    tot = evs[0][0].elapsed_time(evs[-1][3])
    print(f"forward+loss {acc[0] / steps:.2f} ms   backward {acc[1] / steps:.2f} ms   optimizer {acc[2] / steps:.2f} ms"
          f"   (sum {sum(acc) / steps:.2f}; wall per step incl. gaps {tot / steps:.2f})", flush=True)


if __name__ == "__main__":
    main()
