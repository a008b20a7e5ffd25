"""Short-M GEMM routes (the unit decoder's projections: M = target tokens of a batch, a few hundred
rows).  The default is the whole-K small-tile kernel (csrc/gemm_skinny.h); the split-K route (K split
over ~512 workgroups, fused epilogue applied in a fixup pass, include/mms2ut.h splitk_ws) and the
unsplit 128x128 kernel remain behind mms2ut_gemm_set_skinny(0).  Checked against each other on the
same operands: values within fp32-summation-order noise (fp16 outputs: 2e-3 relative L2) and the
dropout masks identical, plus the fp32 torch product for the plain epilogue.  Also: the tall NT tiles
are bit-identical to the 128x128 kernel."""
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _linear(K_, x, W, bias, fixup, epi, aux=None, out2=None, p=0.0, drop=None):
    """K.linear with the split-K fixup on or off (kernels.gemm fixup=)."""
    M, Kd = x.shape
    N = W.shape[0]
    out = torch.empty(M, N, dtype=torch.float16, device=x.device)
    seed, off = drop if p > 0 else (0, 0)
    K_.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, epi=epi, bias=bias, aux=aux,
            ldaux=0 if aux is None else aux.stride(0), out2=out2, ldo2=0 if out2 is None else out2.stride(0),
            p=p, seed=seed, offset=off, ld_rng=N, fixup=fixup)
    return out


ROUTES = (("skinny", 2, True), ("default", 1, True), ("fixup", 0, True), ("unsplit", 0, False))


@pytest.mark.parametrize("M,N,K", [(466, 768, 3072), (466, 3072, 768), (300, 768, 768), (700, 2304, 768),
                                   (129, 768, 3072), (470, 1536, 2560), (1000, 1536, 768), (17, 1004, 768),
                                   (1, 768, 768), (50, 256, 64), (2000, 768, 512), (20, 256, 3072)])
def test_short_m_routes_agree(M, N, K):
    """The routes of a short-M fused-epilogue GEMM on the same operands: the short-M kernel forced
    (mode 2; tile codes 64x64 / 32x64 / 32x32, with and without a K split, all covered), the default
    route table (mode 1), split-K + fixup, and the unsplit 128x128 kernel.  Values agree within fp32-summation-order noise, dropout masks are
    identical (a large positive bias keeps every ReLU open, so the zero pattern IS the mask), and the
    plain epilogue matches the fp32 torch product."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K_ = mm.kernels
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).half()
    b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
    aux = torch.randn(M, N, device="cuda", generator=g).half()
    big = torch.full((N,), 30.0, device="cuda").half()
    c0 = torch.randn(M, N, device="cuda", generator=g).half()
    cases = [("f16", dict(epi=K_.EPI_F16)),
             ("relu_drop_open", dict(epi=K_.EPI_RELU_DROP, p=0.1, drop=(11, 4096), bias=big)),
             ("relu_drop", dict(epi=K_.EPI_RELU_DROP, p=0.1, drop=(11, 4096))),
             ("drop_resid", dict(epi=K_.EPI_DROP_RESID, p=0.1, drop=(5, 0), aux=aux)),
             ("relu_drop_bwd", dict(epi=K_.EPI_RELU_DROP_BWD, p=0.1, drop=(5, 0), aux=aux)),
             ("gelu_drop", dict(epi=K_.EPI_GELU_DROP, p=0.1, drop=(3, 64),
                                out2=torch.empty(M, N, device="cuda", dtype=torch.float16))),
             ("gelu_drop_bwd", dict(epi=K_.EPI_GELU_DROP_BWD, p=0.1, drop=(3, 64), aux=aux)),
             ("f16_acc", dict(epi=K_.EPI_F16_ACC)),
             ("gate", dict(epi=K_.EPI_GATE, aux=torch.randn(M, 2 * N, device="cuda", generator=g).half(),
                           out2=torch.empty(M, N, device="cuda", dtype=torch.float16)))]
    if N % 8:
        cases = [c for c in cases if c[0] != "gate"]
    try:
        for name, kw in cases:
            kw = dict(kw)
            bias = kw.pop("bias", b if kw["epi"] not in (K_.EPI_RELU_DROP_BWD, K_.EPI_GELU_DROP_BWD) else None)
            outs = {}
            for route, skinny, fix in ROUTES:
                K_.call("mms2ut_gemm_set_skinny", skinny)
                o2 = kw.get("out2")
                if o2 is not None:
                    o2.zero_()
                if kw["epi"] == K_.EPI_F16_ACC:
                    out = c0.clone()
                    K_.gemm(x, W, out, M, N, K, lda=K, ldb=K, ldc=N, epi=K_.EPI_F16_ACC, fixup=fix)
                else:
                    out = _linear(K_, x, W, bias, fix, **kw).clone()
                outs[route] = (out, None if o2 is None else o2.clone())
            torch.cuda.synchronize()
            ref, ref2 = outs["unsplit"]
            for route in ("skinny", "default", "fixup"):
                got, got2 = outs[route]
                assert torch.isfinite(got.float()).all(), (name, route)
                assert _rel(got, ref) < 2e-3, (name, route, _rel(got, ref))
                if ref2 is not None:
                    assert _rel(got2, ref2) < 2e-3, (name, route)
                if name == "relu_drop_open":
                    assert torch.equal(got == 0, ref == 0), (name, route)
            if name == "relu_drop_open" and M * N > 10000:
                frac = (outs["skinny"][0] == 0).float().mean().item()
                assert 0.08 < frac < 0.12, frac
            if name == "f16":
                exact = (x.float() @ W.float().t() + b.float())
                assert _rel(outs["skinny"][0], exact) < 2e-3
    finally:
        K_.call("mms2ut_gemm_set_skinny", 1)   # the library default


def test_short_m_split_placement_independent():
    """The short-M kernel's in-kernel split-K hand-off does not depend on where the splits run
    (VERDICT r5 item 2): every split plan (mode 2, fused epilogues, K split 2-12 ways) gives the
    same bits when the splits of every tile are dealt over different XCD groups (bid % 8) as when
    they share one, over repeated launches with a large GEMM running concurrently on a second
    stream.  The recorded hardware XCD ids show the scattered splits really ran on different XCDs."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K_ = mm.kernels
    g = torch.Generator(device="cuda").manual_seed(7)
    xcc = torch.full((1 << 16,), -1, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    bx = torch.randn(8192, 1024, device="cuda", generator=g).half()
    bw = torch.randn(2048, 1024, device="cuda", generator=g).half()
    shapes = [(466, 768, 3072), (129, 768, 3072), (20, 256, 3072), (300, 768, 768), (512, 1024, 2304)]
    try:
        K_.call("mms2ut_gemm_set_skinny", 2)
        for M, N, K in shapes:
            x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
            W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).half()
            b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
            aux = torch.randn(M, N, device="cuda", generator=g).half()
            outs = {}
            for scatter in (0, 1, 0, 1):
                K_.call("mms2ut_gemm_skinny_debug", scatter, xcc.data_ptr() if scatter else 0)
                for rep in range(10):
                    with torch.cuda.stream(side):   # a concurrent grid on the other queue
                        torch.matmul(bx, bw.t())
                    o = _linear(K_, x, W, b, True, K_.EPI_DROP_RESID, aux=aux, p=0.1, drop=(9, 128))
                    prev = outs.setdefault("ref", o.clone())
                    assert torch.equal(o.view(torch.int16), prev.view(torch.int16)), (M, N, K, scatter, rep)
            K_.call("mms2ut_gemm_skinny_debug", 0, 0)
            K_.call("mms2ut_gemm_set_skinny", 0)    # the split-K + fixup route on the same operands
            fix = _linear(K_, x, W, b, True, K_.EPI_DROP_RESID, aux=aux, p=0.1, drop=(9, 128))
            K_.call("mms2ut_gemm_set_skinny", 2)
            torch.cuda.synchronize()
            assert _rel(outs["ref"], fix) < 2e-3, (M, N, K, _rel(outs["ref"], fix))
        K_.call("mms2ut_gemm_skinny_debug", 1, xcc.data_ptr())
        _linear(K_, x, W, b, True, K_.EPI_F16)
        torch.cuda.synchronize()
        ids = xcc[xcc >= 0].cpu()
        assert len(ids) > 0 and int(ids.max()) < 8
        # blocks of different bid % 8 groups (= the splits of one tile when scattered) on different XCDs
        groups = {int(ids[i]) for i in range(min(8, len(ids)))}
        assert len(groups) > 1, groups
    finally:
        K_.call("mms2ut_gemm_skinny_debug", 0, 0)
        K_.call("mms2ut_gemm_set_skinny", 1)


def test_fixup_accumulate_dgrad():
    """dgrad with accumulation (EPI_F16_ACC) at a decoder shape: fixup vs unsplit vs fp32."""
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
        o = base.clone()
        K_.gemm(dy, W, o, M, K, N, a_kc=True, b_kc=False, lda=N, ldb=K, ldc=K, epi=K_.EPI_F16_ACC, fixup=fix)
        outs.append(o)
    torch.cuda.synchronize()
    exact = base.float() + dy.float() @ W.float()
    assert _rel(outs[1], outs[0]) < 2e-3
    assert _rel(outs[1], exact) < 2e-3


# ------------------------------------------------------------------ tall NT tiles
_PP_EPIS = ["F16", "RELU_DROP", "DROP_RESID", "RELU_DROP_BWD", "GATE", "F16_ACC", "GELU_DROP", "GELU_DROP_BWD"]


@pytest.mark.parametrize("M,N,K", [(12000, 768, 768), (12000, 768, 3072), (11001, 768, 2304), (10000, 1000, 640),
                                   (300, 520, 64), (16384, 768, 192)])
def test_tall_gemm_bit_identical(M, N, K):
    """gemm_tall_kernel (96 / 160 / 192 x 128 NT tiles, gemm.hip) against the 128x128 LDS-DMA kernel
    on the same operands: bit-identical for every fused epilogue, incl. ragged M (rows past M in the
    last tile), ragged N, short K, dropout counters; modes 2 / 3 / 5 force 160 / 192 / 96 rows."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mm = pkg()
    K_ = mm.kernels
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 2)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).half()
    b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
    aux = torch.randn(M, 2 * N, device="cuda", generator=g).half()
    c0 = torch.randn(M, N, device="cuda", generator=g).half()
    K_.call("mms2ut_gemm_set_skinny", 0)     # (300, 520, 64) is short-M: keep it on the NT tiles
    try:
        for name in _PP_EPIS:
            epi = getattr(K_, "EPI_" + name)
            outs = []
            for mode in (0, 2, 3, 5):
                K_.call("mms2ut_gemm_set_tall", mode)
                out = c0.clone()
                out2 = torch.zeros(M, N, dtype=torch.float16, device="cuda")
                p = 0.1 if name in ("RELU_DROP", "DROP_RESID", "GELU_DROP", "GELU_DROP_BWD", "RELU_DROP_BWD") else 0.0
                K_.gemm(x, W, out, M, N, K, lda=K, ldb=K, ldc=N, epi=epi, bias=b,
                        aux=aux if name in ("DROP_RESID", "RELU_DROP_BWD", "GATE", "GELU_DROP_BWD") else None,
                        ldaux=2 * N, out2=out2 if name in ("GATE", "GELU_DROP") else None, ldo2=N,
                        p=p, seed=79, offset=7 * N, ld_rng=N, fixup=False)
                outs.append((out, out2))
            torch.cuda.synchronize()
            for mode, (o, o2) in zip((2, 3, 5), outs[1:]):
                assert torch.equal(o.view(torch.int16), outs[0][0].view(torch.int16)), (name, mode)
                assert torch.equal(o2.view(torch.int16), outs[0][1].view(torch.int16)), (name, mode, "out2")
        K_.call("mms2ut_gemm_set_tall", 3)
        got = K_.linear(x, W, b)
        ref = (x.float() @ W.float().t() + b.float())
        assert _rel(got, ref) < 2e-3
    finally:
        K_.call("mms2ut_gemm_set_tall", 1)   # the library defaults
        K_.call("mms2ut_gemm_set_skinny", 1)
