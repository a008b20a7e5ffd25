"""Split-K with a fused-epilogue fixup (include/mms2ut.h splitk_ws): the short-M GEMMs of the unit
decoder (M = target tokens of a batch, a few hundred rows) split K over ~512 workgroups and apply
their epilogue in a second pass.  Checked against the unsplit kernel on the same operands:
values within fp32-summation-order noise (fp16 outputs: 2e-3 relative L2) and the dropout masks
identical (a large positive bias keeps every ReLU open, so the zero pattern IS the mask), plus
the fp32 torch product for the plain epilogue."""
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.mark.parametrize("M,N,K", [(466, 768, 3072), (466, 3072, 768), (300, 768, 768), (700, 2304, 768),
                                   (129, 768, 3072)])
def test_fixup_matches_unsplit(M, N, K):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K_ = mm.kernels
    assert K_._fixup_splits(M, N, K) > 1
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).half()
    b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
    aux = torch.randn(M, N, device="cuda", generator=g).half()
    big = torch.full((N,), 30.0, device="cuda").half()
    cases = [("f16", dict(epi=K_.EPI_F16)),
             ("relu_drop_open", dict(epi=K_.EPI_RELU_DROP, p=0.1, drop=(11, 4096), bias=big)),
             ("relu_drop", dict(epi=K_.EPI_RELU_DROP, p=0.1, drop=(11, 4096))),
             ("drop_resid", dict(epi=K_.EPI_DROP_RESID, p=0.1, drop=(5, 0), aux=aux)),
             ("relu_drop_bwd", dict(epi=K_.EPI_RELU_DROP_BWD, p=0.1, drop=(5, 0), aux=aux)),
             ("gate", dict(epi=K_.EPI_GATE, aux=torch.randn(M, 2 * N, device="cuda", generator=g).half(),
                           out2=torch.empty(M, N, device="cuda", dtype=torch.float16)))]
    if N % 8:
        cases = [c for c in cases if c[0] != "gate"]
    for name, kw in cases:
        kw = dict(kw)
        bias = kw.pop("bias", b if kw["epi"] not in (K_.EPI_RELU_DROP_BWD,) else None)
        outs = []
        for fix in (False, True):
            K_._SPLITK_FIX = fix
            try:
                o2 = kw.get("out2")
                if o2 is not None:
                    o2.zero_()
                outs.append((K_.linear(x, W, bias, **kw).clone(), None if o2 is None else o2.clone()))
            finally:
                K_._SPLITK_FIX = True
        torch.cuda.synchronize()
        (ref, ref2), (got, got2) = outs
        assert _rel(got, ref) < 2e-3, (name, _rel(got, ref))
        if ref2 is not None:
            assert _rel(got2, ref2) < 2e-3, name
        if name == "relu_drop_open":
            assert torch.equal(got == 0, ref == 0), name
            frac = (got == 0).float().mean().item()
            assert 0.08 < frac < 0.12, frac
        if name == "f16":
            exact = (x.float() @ W.float().t() + b.float())
            assert _rel(got, exact) < 2e-3


def test_fixup_accumulate_dgrad():
    """dgrad with accumulation (EPI_F16_ACC) at a decoder shape."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K_ = mm.kernels
    g = torch.Generator(device="cuda").manual_seed(1)
    M, N, K = 466, 3072, 768
    dy = (torch.randn(M, N, device="cuda", generator=g) * 0.1).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).half()
    base = torch.randn(M, K, device="cuda", generator=g).half()
    outs = []
    for fix in (False, True):
        K_._SPLITK_FIX = fix
        try:
            o = base.clone()
            K_.linear_dgrad(dy, W, o, accumulate=True)
            outs.append(o)
        finally:
            K_._SPLITK_FIX = True
    torch.cuda.synchronize()
    exact = base.float() + dy.float() @ W.float()
    assert _rel(outs[1], outs[0]) < 2e-3
    assert _rel(outs[1], exact) < 2e-3


@pytest.mark.parametrize("M,N,K", [(11000, 768, 768), (11000, 768, 3072), (11000, 2304, 768), (12000, 768, 768)])
def test_tail_split_matches_single_launch(M, N, K):
    """A grid that overflows the 512 block slots by a small tail: head rows as usual, tail rows
    split-K + fixup (kernels._tail_split_rows) == one launch, masks identical."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K_ = mm.kernels
    M1 = K_._tail_split_rows(M, N, K)
    assert 0 < M1 < M
    g = torch.Generator(device="cuda").manual_seed(2)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).half()
    aux = torch.randn(M, N, device="cuda", generator=g).half()
    big = torch.full((N,), 30.0, device="cuda").half()
    for name, kw in (("relu_drop_open", dict(epi=K_.EPI_RELU_DROP, p=0.1, drop=(3, 512))),
                     ("drop_resid", dict(epi=K_.EPI_DROP_RESID, p=0.1, drop=(5, 0), aux=aux))):
        outs = []
        tail0 = K_._TAIL_SPLIT
        for tail in (False, True):
            K_._TAIL_SPLIT = tail
            try:
                outs.append(K_.linear(x, W, big, **kw).clone())
            finally:
                K_._TAIL_SPLIT = tail0
        torch.cuda.synchronize()
        assert _rel(outs[1], outs[0]) < 2e-3, name
        assert torch.equal(outs[1][:M1], outs[0][:M1]), name        # the head is the same launch
        if name == "relu_drop_open":
            assert torch.equal(outs[1] == 0, outs[0] == 0)


@pytest.mark.parametrize("M", [4096, 470, 1003])
def test_relu_mask_roundtrip(M):
    """fc1 forward writes the 1-bit ReLU+dropout activity mask (bit n%8 of byte n/8 = out > 0) and
    the fc2 dgrad epilogue reading it is bit-identical to reading the fp16 activation — on the
    LDS-staged fast path, the short-M split-K fixup path and an odd M."""
    K = pkg().kernels
    torch.manual_seed(0)
    F, d = 3072, 768
    x = torch.randn(M, d, device="cuda").half()
    W1 = (0.05 * torch.randn(F, d, device="cuda")).half()
    b1 = torch.randn(F, device="cuda").half()
    mask = K.relu_mask_alloc(M, F, "cuda").fill_(0xAA)
    f1 = K.linear(x, W1, b1, epi=K.EPI_RELU_DROP, p=0.1, drop=(11, 4096), mask=mask)
    assert torch.equal(K.relu_mask_unpack(mask, M, F), f1 > 0)
    f1b = K.linear(x, W1, b1, epi=K.EPI_RELU_DROP, p=0.1, drop=(11, 4096))
    assert torch.equal(f1, f1b)          # writing the mask does not change the activation
    dy = torch.randn(M, d, device="cuda").half()
    W2 = (0.05 * torch.randn(d, F, device="cuda")).half()
    ref = K.linear_dgrad(dy, W2, epi=K.EPI_RELU_DROP_BWD, aux=f1, p=0.1)
    got = K.linear_dgrad(dy, W2, epi=K.EPI_RELU_DROP_BWD, mask=mask, p=0.1)
    assert torch.equal(ref, got)
