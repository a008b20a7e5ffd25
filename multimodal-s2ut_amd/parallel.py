"""Data parallelism over RCCL (torch.distributed backend "nccl" on ROCm = RCCL over xGMI).

Replaces fairseq's DDP wrap (distributed_fairseq_model.py: torch DDP, bucket_cap_mb=25).  The
parameter layout is in backward-completion order (model.param_specs), so the flat fp16 gradient
buffer fills front-to-back during the hand-written backward; the model calls ``ready(offset)``
after each layer and every bucket wholly below ``offset`` is all-reduced (SUM) at once,
asynchronously on RCCL's stream, overlapping the rest of the backward.  Never-used parameters
 live outside the flat buffer, so they are never communicated.  The fairseq per-step
``all_gather_list`` of logging outputs becomes one summed all-reduce of fixed scalars.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """One process per GPU, launched by torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE).
    Returns (rank, world, device index).  MMS2UT_DIST_BACKEND overrides the backend; with more
    local ranks than devices (a gloo rehearsal of the N > 1 path on a one-GPU box) ranks share
    devices round-robin."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev > 0 and local >= ndev:
        if os.environ.get("MMS2UT_DIST_BACKEND", "") != "gloo":
            raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} GPUs (RCCL needs one GPU per rank)")
        local = local % ndev
    if world > 1 and not dist.is_initialized():
        backend = backend or os.environ.get("MMS2UT_DIST_BACKEND") or None
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        kw = {}
        if backend == "nccl" and torch.cuda.is_available():
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


class GradAllReducer:
    """Bucketed, backward-overlapped all-reduce of a flat gradient buffer with torch DDP's
    arithmetic: each bucket is divided by the world size in place, then SUM-all-reduced, so the
    fp16 gradient magnitudes (hence overflow and the loss-scale trajectory) are those of fairseq's
    DDP-averaged gradients; the optimizer's multiply factor carries world/sample_size as fairseq's
    ``multiply_grads(world / sample_size)`` does.  ``acc`` (fp32, optional): gradients accumulated
    over earlier --update-freq micro-batches, added into each bucket right before it is reduced."""

    def __init__(self, grad_flat, bucket_mb=64.0, group=None, prescale=None, merge=None):
        """prescale(bucket, alpha) / merge(bucket, acc_bucket): in-place bucket arithmetic, the HIP
        kernels by default (kernels.scale_f16 / add_f32_to_f16); host-tensor rehearsals of the
        bookkeeping (tests/test_plugins.py, gloo on CPU) pass their own."""
        from . import kernels as K
        self.prescale = prescale or K.scale_f16
        self.merge = merge or (lambda g, a: K.add_f32_to_f16(g, a, g))
        self.grad = grad_flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        n = grad_flat.numel()
        per = max(1, int(bucket_mb * 2 ** 20 // grad_flat.element_size()))
        per = (per + 7) // 8 * 8
        self.bounds = [(a, min(n, a + per)) for a in range(0, n, per)]
        self.acc = None
        self.reset()

    def reset(self):
        self.next = 0
        self.handles = []

    def ready(self, upto):
        if self.world == 1:
            return
        if self.next >= len(self.bounds) or self.bounds[self.next][1] > upto:
            return
        # gradients of a bucket come from both the main stream (LayerNorm/embedding grads) and the
        # weight-gradient side stream: enqueue the collective behind both
        from . import kernels as K
        side = K._Side.stream
        ctx = None
        if side is not None and K._Side.used:
            K.stream_wait(side, torch.cuda.current_stream())
            ctx = torch.cuda.stream(side)
        with (ctx or K._NULLCTX):
            while self.next < len(self.bounds) and self.bounds[self.next][1] <= upto:
                a, b = self.bounds[self.next]
                g = self.grad[a:b]
                if self.acc is not None:
                    self.merge(g, self.acc[a:b])
                self.prescale(g, 1.0 / self.world)
                self.handles.append(dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group,
                                                    async_op=True))
                self.next += 1

    def finish(self):
        if self.world == 1:
            return
        self.ready(self.grad.numel())
        for h in self.handles:
            h.wait()
        self.reset()


class GradNormCheck:
    """fairseq Trainer._check_grad_norms: after the gradient all-reduce every rank's grad norm
    must agree (relative 1e-6).  Runs on device (kernels.grad_norm_check + one [world] fp32
    all-reduce); an inconsistent step is not applied and the optimizer state turns FATAL, which
    the host raises as FloatingPointError at its next read (FP16Adam.stats)."""

    def __init__(self, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.buf = torch.zeros(max(self.world, 1), dtype=torch.float32, device=device)

    def __call__(self, ost):
        from . import kernels as K
        K.grad_norm_check(self.buf, self.world, self.rank, ost, 0)
        if self.world > 1:
            dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group)
        K.grad_norm_check(self.buf, self.world, self.rank, ost, 1)


def all_reduce_scalars(t, group=None):
    """Summed all-reduce of a small fp32 vector (replaces fairseq all_gather_list logging)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
