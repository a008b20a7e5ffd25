"""Trainer: one optimizer update per batch (update-freq 1), fairseq Trainer.train_step semantics.

  zero grads -> fwd (model + LS-CE) -> loss.backward(loss_scale) [hand-written bwd, bucketed RCCL
  all-reduce overlapped] -> sample_size all-reduce -> FP16Optimizer/Adam (device-side overflow skip
  + loss-scale update) -> lr schedule.

fairseq reference: Trainer.train_step (multiply_grads(world/sample_size) after DDP's averaging
== SUM all-reduce then 1/sample_size), FP16Optimizer.clip_grad_norm(10), DynamicLossScaler.
"""
import os

import torch

from . import kernels as K
from . import runtime
from .optim import FP16Adam
from .parallel import GradAllReducer, all_reduce_scalars


class Trainer:
    def __init__(self, model, lr=5e-4, betas=(0.9, 0.98), clip_norm=10.0, warmup_updates=10000,
                 warmup_init_lr=1e-7, init_scale=128.0, bucket_mb=64.0, world_size=1):
        self.model = model
        self.cfg = model.cfg
        self.opt = FP16Adam(model.params, lr=lr, betas=betas, clip_norm=clip_norm, init_scale=init_scale,
                            world_size=world_size, warmup_updates=warmup_updates,
                            warmup_init_lr=warmup_init_lr)
        self.reducer = GradAllReducer(model.params.grad, bucket_mb) if world_size > 1 else None
        self.world = world_size
        self.log = torch.zeros(4, dtype=torch.float32, device=model.params.flat.device)
        # The step's critical path (forward, dgrad chain, optimizer) runs on a high-priority stream
        # so the hardware dispatcher prefers its workgroups over the weight-gradient side stream's
        # (lowest priority), which only fills the CUs the critical path leaves idle.
        self.stream = None
        if os.environ.get("MMS2UT_STREAM_PRIO", "1") != "0" and model.params.flat.is_cuda:
            self.stream = torch.cuda.Stream(device=model.params.flat.device, priority=-100)
            if K._Side.stream is None:
                K._Side.stream = K.make_side_stream(model.params.flat.device)
                K._Side.ptr = K._Side.stream.cuda_stream

    def train_step(self, batch):
        if self.stream is None:
            return self._train_step(batch)
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            log = self._train_step(batch)
        cur.wait_stream(self.stream)
        return log

    def _train_step(self, batch):
        cfg = self.cfg
        m = self.model
        m.train()
        if self.reducer is not None:
            self.reducer.reset()
            m.grad_ready_hook = self.reducer.ready
        logits = runtime.model_logits(m, batch)
        # zeroed after the forward: by then every deferred optimizer chunk of the previous step
        # (which reads the gradients) has been waited for (ParamStore.await_group)
        m.params.await_all()
        if not getattr(m.params, "grad_zeroed", False):
            m.params.grad.zero_()
        m.params.grad_zeroed = False
        loss, nll = runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"],
                                              cfg["label_smoothing"], cfg["padding_idx"])
        del logits
        loss.backward(self.opt.loss_scale())
        m.grad_ready_hook = None
        if self.reducer is not None:
            self.reducer.finish()
        # logging / sample-size sync: [loss, nll, ntokens, nsentences] summed over ranks
        self.log[0] = loss.detach()
        self.log[1] = nll.detach()
        # fill_ takes the scalar as a kernel argument (item assignment would be a blocking H2D copy)
        self.log[2].fill_(float(batch.ntokens))
        self.log[3].fill_(float(batch.nsentences))
        all_reduce_scalars(self.log)
        self.opt.step(self.log[2:3])
        return self.log

    def valid_step(self, batch):
        m = self.model
        m.eval()
        with torch.no_grad():
            logits = runtime.model_logits(m, batch)
            loss, nll = runtime.label_smoothed_ce(logits, batch.target, self.cfg["vocab_size"],
                                                  self.cfg["label_smoothing"], self.cfg["padding_idx"])
        m.train()
        return loss, nll
