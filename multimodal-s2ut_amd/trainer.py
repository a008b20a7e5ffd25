"""Trainer: one optimizer update per ``update_freq`` micro-batches, fairseq Trainer.train_step
semantics.

  per micro-batch: fwd (model + LS-CE) -> loss.backward(loss_scale) [hand-written bwd]
  gradients of micro-batches 1..n-1 accumulate into an fp32 buffer; the last micro-batch's
  backward adds it bucket by bucket just before the bucketed RCCL all-reduce (overlapped with the
  backward) -> scalar all-reduce (loss, nll, ntokens, ...) -> grad norm -> cross-rank grad-norm
  consistency check -> FP16Optimizer/Adam (device-side overflow skip + loss-scale update) -> lr.

fairseq reference: Trainer.train_step (DDP no_sync on all but the last micro-batch; DDP averages
gradients, then multiply_grads(world/sample_size) with sample_size summed over micro-batches and
ranks), FP16Optimizer.clip_grad_norm(10), DynamicLossScaler (scale window 2^14/world/update_freq),
Trainer._check_grad_norms.

HIP-graph mode (``graph=True``, world size 1): the whole update -- forward, hand-written backward
(both streams), loss scaling, grad norm and the Adam update -- is captured once per (micro-batch
set, modality-dropout branch) with torch.cuda.graph and replayed, so a step costs one graph launch
instead of ~2000 kernel launches issued from Python.  What varies between replays lives on the
device: the dropout seed (a device step counter every dropout kernel adds to its seed,
include/mms2ut.h mms2ut_bind_step_seed), the loss scale, step count and learning rate (optimizer
state vector).  The modality-dropout draws (two numpy draws per forward, as the reference) are
made before the step and select the graph.  Batches must stay resident (the graph bakes their
device pointers): the first step on a new batch runs eagerly, then captures.

Buffer access: the Adam update runs deferred on the side stream (optim.FP16Adam.step).  Call ``trainer.sync()`` (or ``model.params.await_all()``) before reading
``params.flat`` / ``params.grad`` / ``opt.master`` directly after a step; ``state_dict``,
``opt.stats`` and the next forward wait by themselves.
"""

import numpy as np
import torch

from . import kernels as K
from . import runtime
from .optim import FP16Adam
from .parallel import GradAllReducer, GradNormCheck, all_reduce_scalars

# log slots (all-reduced SUM over ranks every step)
LOG_LOSS, LOG_NLL, LOG_NTOKENS, LOG_NSENT, LOG_SS_OVER_WORLD = range(5)
# per-update increment of the device step seed (odd 64-bit golden-ratio constant)
STEP_SEED_INC = 0x9E3779B97F4A7C15


class _ScriptedDraws:
    """Stands in for numpy's global stream inside the model while a graph-mode step runs: the
    step's modality-dropout draws are made up front (they select the graph) and handed out here."""

    def __init__(self):
        self.vals = []

    def random(self):
        if not self.vals:
            raise RuntimeError("graph-mode trainer: unexpected modality-dropout draw")
        return self.vals.pop(0)


class Trainer:
    def __init__(self, model, lr=5e-4, betas=(0.9, 0.98), clip_norm=10.0, warmup_updates=10000,
                 warmup_init_lr=1e-7, init_scale=128.0, bucket_mb=64.0, world_size=1, update_freq=1,
                 graph=False, device_seed=None, max_graphs=64):
        self.model = model
        self.cfg = model.cfg
        self.update_freq = int(update_freq)
        if self.update_freq < 1:
            raise ValueError("update_freq must be >= 1")
        self.opt = FP16Adam(model.params, lr=lr, betas=betas, clip_norm=clip_norm, init_scale=init_scale,
                            world_size=world_size, update_freq=self.update_freq,
                            warmup_updates=warmup_updates, warmup_init_lr=warmup_init_lr)
        self.reducer = GradAllReducer(model.params.grad, bucket_mb) if world_size > 1 else None
        self.norm_check = GradNormCheck(model.params.flat.device) if world_size > 1 else None
        self.world = world_size
        self.acc = None   # fp32 gradient accumulator (update_freq > 1), allocated on first use
        self.log = torch.zeros(5, dtype=torch.float32, device=model.params.flat.device)
        self.grad_tap = None   # optional callable(flat fp16 grad) run right before the optimizer (tests)
        # The step's critical path (forward, dgrad chain, optimizer) runs on a high-priority stream
        # so the hardware dispatcher prefers its workgroups over the weight-gradient side stream's
        # (lowest priority), which only fills the CUs the critical path leaves idle.
        self.stream = None
        if model.params.flat.is_cuda:
            self.stream = K.make_stream(model.params.flat.device, -100)
            if K._Side.stream is None:
                K._Side.stream = K.make_side_stream(model.params.flat.device)
                K._Side.ptr = K._Side.stream.cuda_stream
        # device step seed: every update draws its dropout masks from (base seed + step * INC, offsets
        # from 0); graph mode needs it (a replay cannot change a kernel's seed argument), eager mode
        # can opt in (bit-identical to graph mode)
        self.graph_mode = bool(graph)
        self.device_seed = self.graph_mode if device_seed is None else bool(device_seed)
        if self.graph_mode and not self.device_seed:
            raise ValueError("graph mode needs the device step seed")
        if self.device_seed:
            self.seed_delta = torch.zeros(1, dtype=torch.int64, device=model.params.flat.device)
            self.seed_base = model.drop.seed
        if self.graph_mode:
            if world_size != 1 or self.stream is None:
                raise ValueError("graph mode: single process on a GPU (world size 1) only")
            self.opt.defer = False        # no cross-step event handoff: each replay is self-contained
            self.graphs = {}
            self.max_graphs = int(max_graphs)
            self.pool = torch.cuda.graph_pool_handle()
            self.draws = _ScriptedDraws()
            model.np_rng = self.draws
            # buffers baked into a captured graph must outlive it: regrown scratch / tables are retired,
            # never freed
            K._Side.retain = True
            model.retain_tables = True

    def sync(self):
        """Wait (on the current stream) for every deferred optimizer chunk of the last step."""
        self.model.params.await_all()

    def train_step(self, batches, prologue=None, eager=False, draws=None):
        """batches: one runtime.DeviceBatch or a list of ``update_freq`` micro-batches (fairseq's
        ``samples``).  Returns the device log [loss, nll, ntokens, nsentences, ntokens/world]
        summed over micro-batches and ranks.

        prologue: optional callable run at the start of the step (in graph mode it is captured
        with it, e.g. the fbank front end refreshing ``batch.src``).  eager=True (graph mode): run
        this step without capturing or replaying (e.g. for per-kernel timing).  draws (graph mode):
        explicit (modality, audio) draw pairs per micro-batch instead of numpy's stream (to capture
        a chosen modality-dropout branch ahead of time)."""
        if not isinstance(batches, (list, tuple)):
            batches = [batches]
        if len(batches) != self.update_freq:
            raise ValueError(f"train_step: {len(batches)} micro-batches for update_freq {self.update_freq}")
        if self.device_seed:
            K.bind_step_seed(self.seed_delta)
        if self.graph_mode:
            return self._graph_step(batches, prologue, eager, draws)
        if prologue is not None:
            prologue()
        if self.stream is None:
            return self._train_step(batches)
        cur = torch.cuda.current_stream()
        K.stream_wait(self.stream, cur)
        with torch.cuda.stream(self.stream):
            log = self._train_step(batches)
        # the hand-back to the caller's stream is where the host reads the loss or starts copies /
        # peer collectives: a system-scope event (torch's), one per step; the internal fork / joins
        # stay on device-scope events
        cur.wait_stream(self.stream)
        return log

    def _graph_step(self, batches, prologue, eager, draws):
        m, cfg = self.model, self.cfg
        branches = []
        for i, b in enumerate(batches):   # the reference's two draws per training forward with images
            if cfg["fusion"] and b.imgs is not None:
                mod_p, aud_p = draws[i] if draws is not None else (np.random.random(), np.random.random())
                self.draws.vals += [mod_p, aud_p]
                branches.append(None if not mod_p < cfg["modality_dropout"] else
                                "audio" if aud_p < cfg["audio_dropout"] else "image")
            else:
                branches.append(None)
        key = (tuple(id(b) for b in batches), tuple(branches))
        cur = torch.cuda.current_stream()
        K.stream_wait(self.stream, cur)
        entry = None if eager else self.graphs.get(key)
        if entry is None:
            # first time: a real eager step (lazy allocations, table growth), then capture the same
            # step (capture executes nothing) with the same draws
            vals = list(self.draws.vals)
            with torch.cuda.stream(self.stream):
                if prologue is not None:
                    prologue()
                log = self._train_step(batches)
            if not eager:
                if len(self.graphs) >= self.max_graphs:
                    # each graph pins its batches and every scratch buffer it baked in: graph mode is
                    # for a fixed resident batch set (the bench), not a stream of fresh batches
                    raise RuntimeError(f"graph mode: more than {self.max_graphs} distinct (batch set, modality "
                                       "branch) keys; use eager mode for streamed batches")
                self.draws.vals = vals
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.pool, stream=self.stream):
                    if prologue is not None:
                        prologue()
                    self._train_step(batches)
                self.graphs[key] = (g, list(batches))    # keep the batches (their pointers are baked)
            self.draws.vals = []
        else:
            self.draws.vals = []
            with torch.cuda.stream(self.stream):
                entry[0].replay()
            log = self.log
        cur.wait_stream(self.stream)   # system-scope hand-back (see train_step)
        return log

    def _train_step(self, batches):
        cfg = self.cfg
        m = self.model
        m.train()
        n = len(batches)
        if self.device_seed:
            K.step_seed_advance(self.seed_delta, STEP_SEED_INC)
            m.drop.reset(self.seed_base)
        if n > 1 and self.acc is None:
            self.acc = torch.zeros(m.params.numel, dtype=torch.float32, device=m.params.flat.device)
        ntok = sum(int(b.ntokens) for b in batches)
        # the step log in one launch: loss / nll accumulate into it (the LS-CE kernel adds each
        # micro-batch's sums), ntokens / nsentences / sample size per world are known up front
        K.set_f32(self.log, [0.0, 0.0, float(ntok), float(sum(int(b.nsentences) for b in batches)),
                             float(ntok) / self.world])
        for i, batch in enumerate(batches):
            last = i == n - 1
            if self.reducer is not None and last:
                self.reducer.reset()
                self.reducer.acc = self.acc if n > 1 else None
                m.grad_ready_hook = self.reducer.ready
            logits, aux = runtime.model_outputs(m, batch)
            # The hand-written backward defines every gradient outright: each parameter's gradient
            # is written (not added to) by its backward, or zeroed where a branch skips it
            # (model._zero_grads), so the flat buffer is never cleared as a whole (that fill moved
            # 301 MB per step).  By now every deferred optimizer chunk of the previous step (which
            # reads the gradients) has been waited for (ParamStore.await_group).
            m.params.await_all()
            if m.params.zero_each_step:
                m.params.grad.zero_()
            loss, nll = runtime.label_smoothed_ce(logits, batch.target, cfg["vocab_size"],
                                                  cfg["label_smoothing"], cfg["padding_idx"],
                                                  acc=self.log[LOG_LOSS:LOG_NLL + 1])
            del logits
            # multitask heads: loss + sum_t weight_t * loss_t (fairseq MultitaskCriterion); the
            # logged loss stays the main one (fairseq logs multitask losses separately)
            (loss + aux if aux is not None else loss).backward(self.opt.loss_scale())
            m.grad_ready_hook = None
            if n > 1:
                if i == 0:
                    self.acc.zero_()
                if not last:
                    K.accum_f16_f32(self.acc, m.params.grad)
                elif self.reducer is None:
                    K.add_f32_to_f16(m.params.grad, self.acc, m.params.grad)
        if self.reducer is not None:
            self.reducer.finish()
            self.reducer.acc = None
        # logging / sample-size sync: the log (set at the step start) summed over ranks
        all_reduce_scalars(self.log)
        if self.grad_tap is not None:
            # the final (reduced, accumulated) fp16 gradient, in stream order before the optimizer
            # consumes and (deferred path) zeroes it
            self.grad_tap(m.params.grad)
        # DDP-averaged gradients (sum / world): multiply factor world / (scale * sample_size)
        self.opt.step(self.log[LOG_SS_OVER_WORLD:LOG_SS_OVER_WORLD + 1], check=self.norm_check)
        return self.log

    def valid_step(self, batch):
        m = self.model
        m.eval()
        with torch.no_grad():
            logits, aux = runtime.model_outputs(m, batch)
            loss, nll = runtime.label_smoothed_ce(logits, batch.target, self.cfg["vocab_size"],
                                                  self.cfg["label_smoothing"], self.cfg["padding_idx"])
        m.train()
        return loss, nll

    # ------------------------------------------------------------------ checkpoints
    def completed_updates(self):
        """fairseq's num_updates: optimizer steps that were applied (fp16-overflow skips excluded),
        read from the device state (a host sync)."""
        self.sync()
        return int(self.opt.ost[K.OST_STEP].item())

    def state_dict(self):
        """fairseq checkpoint layout (checkpoint_utils.save_checkpoint): model (fairseq keys),
        last_optimizer_state (fp32 master / Adam moments / device optimizer state vector, plus
        FP16Optimizer's ``loss_scale``), optimizer_history, extra_state (num_updates and the
        train iterator position ``train_iterator`` = {epoch, iterations_in_epoch})."""
        self.sync()
        o = self.opt
        n = int(o.ost[K.OST_STEP].item())
        pos = dict(getattr(self, "position", None) or {"epoch": 1, "iterations_in_epoch": 0})
        return {"model": {k: v.detach().cpu() for k, v in self.model.params.state_dict().items()},
                "last_optimizer_state": {"master": o.master.cpu(), "exp_avg": o.exp_avg.cpu(),
                                         "exp_avg_sq": o.exp_avg_sq.cpu(), "ost": o.ost.cpu(),
                                         "loss_scale": float(o.ost[K.OST_LOSS_SCALE].item())},
                "optimizer_history": [{"criterion_name": "SpeechToUnitMultitaskTaskCriterion",
                                       "optimizer_name": "FP16Optimizer",
                                       "lr_scheduler_state": {"best": None}, "num_updates": n}],
                "extra_state": {"num_updates": n, "train_iterator": dict(pos, shuffle=True)}}

    def load_state_dict(self, ckpt):
        """Our own checkpoints restore the exact optimizer state.  A checkpoint written by fairseq
        (its FP16Optimizer state has a different layout: per-parameter-group Adam state over
        fairseq's flattened fp32 params) restores the weights, re-derives the fp32 master from them
        (FP16Optimizer's behaviour with --reset-optimizer), starts fresh Adam moments and keeps
        num_updates (lr schedule position) and the loss scale when the file records them."""
        self.sync()
        self.model.params.load_state_dict({k: v for k, v in ckpt["model"].items()
                                           if k != "decoder.output_projection.weight"})
        o, s = self.opt, ckpt.get("last_optimizer_state")
        ours = isinstance(s, dict) and all(k in s for k in ("master", "exp_avg", "exp_avg_sq", "ost"))
        if ours:
            for name in ("master", "exp_avg", "exp_avg_sq", "ost"):
                getattr(o, name).copy_(s[name])
            return
        o.resync_master()
        o.exp_avg.zero_()
        o.exp_avg_sq.zero_()
        hist = ckpt.get("optimizer_history") or [{}]
        n = (ckpt.get("extra_state") or {}).get("num_updates", hist[-1].get("num_updates", 0))
        o.ost[K.OST_STEP] = float(n or 0)
        if isinstance(s, dict) and s.get("loss_scale") is not None:
            o.ost[K.OST_LOSS_SCALE] = float(s["loss_scale"])
