"""fairseq FP16Optimizer + Adam + inverse_sqrt, MI355X-native and device-resident.

Flat fp32 master / exp_avg / exp_avg_sq mirror the flat fp16 parameter buffer.  Per step:
grad_sqnorm -> grad_norm_finalize (multiply factor 1/(loss_scale*sample_size), overflow flag) ->
optim_prepare (Adam step count + step size, clip coefficient, DynamicLossScaler) -> adam.  No host
synchronisation: the loss scale the next backward uses is read from device memory.

Reference semantics (fairseq, invoked by textless/1_train.sh:105-125):
  --optimizer adam --adam-betas '(0.9,0.98)' --clip-norm 10.0 --lr-scheduler inverse_sqrt
  --warmup-init-lr 1e-7 --warmup-updates 10000 --fp16 (init scale 128, scale window 2^14/world).
"""
import math

import torch

from . import kernels as K


class FP16Adam:
    def __init__(self, params, lr=5e-4, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.0, clip_norm=10.0,
                 init_scale=128.0, scale_window=None, min_loss_scale=1e-4, world_size=1, update_freq=1,
                 warmup_updates=10000, warmup_init_lr=1e-7):
        self.params = params
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.clip = clip_norm
        self.master = params.flat.float()
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self.scale_window = scale_window or max(1, int(2 ** 14 / world_size / update_freq))
        self.min_loss_scale = min_loss_scale
        self.warmup_updates, self.warmup_init_lr = warmup_updates, warmup_init_lr
        self.num_updates = 0  # for get_lr() only; the step counts updates on device (ost[OST_STEP])
        ost = torch.zeros(K.OST_SIZE, dtype=torch.float32)
        ost[K.OST_LOSS_SCALE] = init_scale
        ost[K.OST_LAST_OVERFLOW] = -1.0
        ost[K.OST_CLIP_COEF] = 1.0
        self.ost = ost.to(params.flat.device)
        self.defer = True   # False: one Adam launch in stream order (tests compare both)
        self._events = {}   # group -> K.DevEvent re-recorded by each deferred update

    def resync_master(self):
        """After loading fp16 weights: master := fp32 copy of the fp16 params."""
        self.master.copy_(self.params.flat)

    def loss_scale(self):
        """0-dim device tensor: the gradient fed to loss.backward()."""
        return self.ost[K.OST_LOSS_SCALE]

    def get_lr(self):
        """fairseq inverse_sqrt schedule at ``num_updates`` (host restatement; the step itself
        evaluates the same schedule on device at the count of completed, non-skipped updates)."""
        if self.warmup_updates > 0 and self.num_updates < self.warmup_updates:
            step = (self.lr - self.warmup_init_lr) / self.warmup_updates
            return self.warmup_init_lr + self.num_updates * step
        wu = max(self.warmup_updates, 1)
        return self.lr * math.sqrt(wu) * max(self.num_updates, 1) ** -0.5

    def step(self, sample_size, check=None):
        """sample_size: device fp32 tensor [1] (all-reduced ntokens).

        The global part (grad norm, clip factor, overflow / loss-scale logic) runs on the current
        stream.  The Adam update itself is deferred: it is enqueued on the side stream in chunks,
        one per forward-consumption group of the parameter layout (subsampler, encoder layer 0, ...),
        each recording an event that the next forward waits on right before it reads that group
        (ParamStore.await_group), so the HBM-bound update can overlap the next step's first
        layers (default; 1-1.5 % faster step, bit-identical).  defer = False runs one launch in
        stream order instead."""
        b1, b2 = self.betas
        K.grad_norm(self.params.grad, self.ost, sample_size)
        if check is not None:
            check(self.ost)      # parallel.GradNormCheck: cross-rank grad-norm consistency
        K.optim_prepare(self.ost, self.lr, self.warmup_init_lr, self.warmup_updates, b1, b2, self.clip,
                        self.scale_window, self.min_loss_scale)
        ps = self.params
        if not (self.defer and ps.flat.is_cuda and hasattr(ps, "groups")):
            K.adam(ps.flat, ps.grad, self.master, self.exp_avg, self.exp_avg_sq, self.ost, b1, b2, self.eps,
                   self.wd)
            return
        ps.await_all()  # the previous step's chunks (normally already awaited by the forward)
        side = K.side_stream(ps.flat.device)
        K.stream_wait(side, torch.cuda.current_stream(ps.flat.device))
        with torch.cuda.stream(side):
            for grp, a, b in ps.groups:
                K.adam(ps.flat[a:b], ps.grad[a:b], self.master[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b],
                       self.ost, b1, b2, self.eps, self.wd)
                ev = self._events.get(grp)
                if ev is None:
                    ev = self._events[grp] = K.DevEvent()
                ps.pending[grp] = ev.record(side)

    def check_fatal(self, st=None):
        """Raise fairseq's FloatingPointError if the device state turned FATAL (sticky: an
        inconsistent grad norm across ranks, Trainer._check_grad_norms, or the minimum loss scale
        reached, DynamicLossScaler).  The state vector is identical on every rank, so every rank
        calling this at the same step raises together."""
        st = st or self.stats()
        if st["inconsistent"]:
            raise FloatingPointError("Fatal error: gradients are inconsistent between workers "
                                     "(fairseq Trainer._check_grad_norms)")
        if st["fatal"]:
            raise FloatingPointError(f"Minimum loss scale reached ({self.min_loss_scale}). Your loss is probably "
                                     "exploding. Try lowering the learning rate, using gradient clipping or "
                                     "increasing the batch size.")
        return st

    def stats(self):
        if hasattr(self.params, "await_all"):
            self.params.await_all()
        o = self.ost.cpu()
        return {"gnorm": float(o[K.OST_GNORM]), "overflow": bool(o[K.OST_OVERFLOW]),
                "loss_scale": float(o[K.OST_LOSS_SCALE]), "step": int(o[K.OST_STEP]),
                "fatal": bool(o[K.OST_FATAL]), "lr": float(o[K.OST_LR]),
                "inconsistent": bool(o[K.OST_INCONSISTENT])}
