"""GPU: device-resident FP16Optimizer/Adam/DynamicLossScaler/inverse_sqrt (optim.py + loss_optim.hip)
against the oracle restatement of fairseq's (oracle/ref_model.py: fp16_optimizer_step,
DynamicLossScaler, inverse_sqrt_lr) over several updates: overflow skip, loss-scale halving and
growth, clipping, warmup->decay.  Master weights: relative error < 1e-5; fp16 params: within 1 ulp."""
import pytest
import torch

from conftest import pkg
from oracle import ref_model as R

pytestmark = pytest.mark.gpu


class _Params:
    def __init__(self, n, dev):
        g = torch.Generator().manual_seed(0)
        self.flat = (torch.randn(n, generator=g) * 0.05).half().to(dev)
        self.grad = torch.zeros(n, dtype=torch.float16, device=dev)


@pytest.mark.parametrize("clip", [10.0, 0.05])
def test_fp16_adam_matches_fairseq_restatement(clip):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    dev = torch.device("cuda")
    n = 1_000_003
    P = _Params(n, dev)
    kw = dict(lr=1e-3, betas=(0.9, 0.98), clip_norm=clip, init_scale=128.0, scale_window=2,
              warmup_updates=3, warmup_init_lr=1e-7)
    opt = mm.optim.FP16Adam(P, **kw)
    master = P.flat.float().cpu()
    ea, eas = torch.zeros(n), torch.zeros(n)
    scaler = R.DynamicLossScaler(128.0, scale_window=2)
    done = 0
    gen = torch.Generator().manual_seed(1)
    for it in range(7):
        ss = 1000.0 + 17 * it
        g = (torch.randn(n, generator=gen) * 3e-3 * scaler.loss_scale * ss / 1000).half()
        if it == 2:
            g[12345] = float("inf")  # fp16 overflow in backward
        P.grad.copy_(g.to(dev))
        opt.step(torch.tensor([ss], device=dev))
        st = opt.stats()
        lr = R.inverse_sqrt_lr(done, 1e-3, 3, 1e-7)
        norm, overflow = R.fp16_optimizer_step([master], [g], [(ea, eas)], done + 1, lr,
                                               1.0 / (scaler.loss_scale * ss), clip_norm=clip)
        assert st["overflow"] == overflow, it
        if overflow:
            scaler.overflow()
        else:
            done += 1
            scaler.update()
            assert abs(st["gnorm"] - norm) <= 1e-4 * norm, (it, st["gnorm"], norm)
            assert abs(st["lr"] - lr) <= 1e-6 * lr
        assert st["loss_scale"] == scaler.loss_scale, (it, st["loss_scale"], scaler.loss_scale)
        assert st["step"] == done
        m = opt.master.cpu()
        err = ((m - master).norm() / master.norm()).item()
        assert err < 1e-5, (it, err)
        p16 = P.flat.cpu().float()
        assert torch.allclose(p16, master.half().float(), rtol=1e-3, atol=1e-7), it


def test_fatal_state_is_sticky():
    """an inconsistent grad norm across ranks (Trainer._check_grad_norms) in a step the
    host does not read makes the device state FATAL for good: that step and every later one apply
    no update, and the next host check raises FloatingPointError (on every rank: the state vector
    is identical on all of them)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K = mm.kernels
    dev = torch.device("cuda")
    P = _Params(4096, dev)
    opt = mm.optim.FP16Adam(P, lr=1e-3, warmup_updates=0, init_scale=1.0)
    ss = torch.tensor([100.0], device=dev)
    P.grad.fill_(0.01)
    opt.step(ss)
    assert opt.check_fatal()["step"] == 1
    m0 = opt.master.clone()
    buf = torch.tensor([1.0, 2.0], device=dev)      # two ranks' norms that disagree
    opt.step(ss, check=lambda ost: K.grad_norm_check(buf, 2, 0, ost, 1))
    opt.step(ss)                                    # a clean step later: still no update
    torch.cuda.synchronize()
    assert torch.equal(opt.master, m0)
    st = opt.stats()
    assert st["inconsistent"] and st["fatal"] and st["step"] == 1
    with pytest.raises(FloatingPointError, match="inconsistent"):
        opt.check_fatal()
