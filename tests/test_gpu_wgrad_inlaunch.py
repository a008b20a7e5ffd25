"""In-launch split-K reduction of the weight-gradient GEMM (gemm.hip splitk_inlaunch_reduce): the
last split of every tile sums the fp32 slabs in split order, so dW and db are bit-identical to the
separate splitk_reduce(_bias) launch; the per-tile arrival counters are back at zero after every
launch (so the next launch on the stream starts clean), on the main and on the side stream."""
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K_,bias", [(5000, 96, 200, False), (10000, 768, 768, True),
                                         (3000, 3072, 768, True), (777, 520, 1000, True),
                                         (12000, 768, 2304, False)])
@pytest.mark.parametrize("side", [False, True])
def test_inlaunch_matches_reduce_kernel(M, N, K_, bias, side):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K = mm.kernels
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(M, N, device="cuda", generator=g).half()
    x = torch.randn(M, K_, device="cuda", generator=g).half()
    outs = []
    red0 = K._INLAUNCH_RED
    try:
        for inl in (False, True, True):          # the second in-launch pass reuses the counters
            K._INLAUNCH_RED = inl
            dW = torch.full((N, K_), 3.0, dtype=torch.float16, device="cuda")
            db = torch.full((N,), 7.0, dtype=torch.float16, device="cuda") if bias else None
            K.linear_wgrad(dy, x, dW, db=db, side=side)
            K.side_join()
            torch.cuda.synchronize()
            outs.append((dW.clone(), None if db is None else db.clone()))
    finally:
        K._INLAUNCH_RED = red0
    for dW, db in outs[1:]:
        assert torch.equal(dW, outs[0][0])
        if bias:
            assert torch.equal(db, outs[0][1])
    ref = dy.float().t() @ x.float()
    assert ((outs[1][0].float() - ref).norm() / ref.norm()).item() < 2e-3
    for buf in K._RED_CNT.values():
        assert int(buf.abs().sum().item()) == 0
