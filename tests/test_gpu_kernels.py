"""GPU: HIP kernels vs plain PyTorch fp32 references (floating-point kernels), via the C-ABI."""
import math

import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg().kernels


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _mat(rows, cols, ld=None, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    ld = ld or cols
    buf = torch.randn(rows, ld, generator=g, device="cuda").half()
    return buf[:, :cols]


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K_", [(130, 200, 104), (257, 96, 768), (64, 1004, 72), (1, 8, 8), (136, 24, 17)])
def test_gemm_layouts(K, a_kc, b_kc, M, N, K_):
    r8 = lambda x: (x + 7) // 8 * 8
    A = _mat(M, K_, ld=r8(K_), seed=1) if a_kc else _mat(K_, M, ld=r8(M), seed=1)
    B = _mat(N, K_, ld=r8(K_), seed=2) if b_kc else _mat(K_, N, ld=r8(N), seed=2)
    Af = A.float() if a_kc else A.float().t()
    Bf = B.float() if b_kc else B.float().t()
    ref = Af @ Bf.t()
    ldc = r8(N)
    C = torch.zeros(M, ldc, dtype=torch.float16, device="cuda")
    K.gemm(A, B, C, M, N, K_, a_kc=a_kc, b_kc=b_kc, lda=A.stride(0), ldb=B.stride(0), ldc=ldc)
    torch.cuda.synchronize()
    assert rel(C[:, :N], ref) < 2e-3


def test_gemm_identity_asymmetric(K):
    # A = I with asymmetric B catches a transposed C-write (guide §3)
    n = 128
    A = torch.eye(n, device="cuda").half()
    B = (torch.arange(n * n, device="cuda").view(n, n) % 97).half()
    C = torch.empty(n, n, dtype=torch.float16, device="cuda")
    K.gemm(A, B, C, n, n, n, lda=n, ldb=n, ldc=n)   # C = A B^T (B is [N, K])
    torch.cuda.synchronize()
    assert torch.equal(C, B.t().contiguous())
    K.gemm(A, B, C, n, n, n, b_kc=False, lda=n, ldb=n, ldc=n)  # B as [K, N] -> C = A B
    torch.cuda.synchronize()
    assert torch.equal(C, B)


def test_gemm_batched_strided_alpha(K):
    Bt, H, T, hd = 3, 4, 37, 64
    d = H * hd
    qkv = torch.randn(Bt * T, 3 * d, device="cuda").half()
    ldS = 40
    S = torch.zeros(Bt * H * T * ldS, dtype=torch.float16, device="cuda")
    K.gemm(qkv, qkv[:, d:], S, T, T, hd, lda=3 * d, ldb=3 * d, ldc=ldS, batch=Bt * H, bdiv=H,
           sA=(T * 3 * d, hd), sB=(T * 3 * d, hd), sC=(H * T * ldS, T * ldS), alpha=0.125)
    torch.cuda.synchronize()
    q = qkv[:, :d].float().view(Bt, T, H, hd).permute(0, 2, 1, 3)
    k = qkv[:, d:2 * d].float().view(Bt, T, H, hd).permute(0, 2, 1, 3)
    ref = 0.125 * q @ k.transpose(-1, -2)
    got = S.view(Bt, H, T, ldS)[..., :T]
    assert rel(got, ref) < 2e-3


def test_gemm_epilogues(K):
    M, N, K_ = 300, 256, 192
    x = torch.randn(M, K_, device="cuda").half()
    W = (0.05 * torch.randn(N, K_, device="cuda")).half()
    b = torch.randn(N, device="cuda").half()
    res = torch.randn(M, N, device="cuda").half()
    pre = x.float() @ W.float().t() + b.float()
    y = K.linear(x, W, b, epi=K.EPI_RELU_DROP)
    assert rel(y, pre.relu()) < 2e-3
    y = K.linear(x, W, b, epi=K.EPI_DROP_RESID, aux=res)
    assert rel(y, pre + res.float()) < 2e-3
    # dropout: replay the mask through the C-ABI
    seed, off = 1234, 4096
    y = K.linear(x, W, b, epi=K.EPI_RELU_DROP, p=0.25, drop=(seed, off))
    m = K.dropout_mask(M * N, 0.25, seed, off, "cuda").view(M, N).float()
    assert rel(y, pre.relu() * m / 0.75) < 2e-3
    assert 0.70 < m.mean().item() < 0.80
    # gate
    merge = torch.randn(M, 2 * N, device="cuda").half()
    Wg = (0.05 * torch.randn(N, 2 * N, device="cuda")).half()
    g = torch.empty(M, N, dtype=torch.float16, device="cuda")
    out = K.linear(merge, Wg, b, epi=K.EPI_GATE, aux=merge, out2=g)
    gr = torch.sigmoid(merge.float() @ Wg.float().t() + b.float())
    o, t = merge[:, :N].float(), merge[:, N:].float()
    torch.cuda.synchronize()
    assert rel(g, gr) < 2e-3
    assert rel(out, (1 - gr) * t + gr * o) < 2e-3


@pytest.mark.parametrize("M,N,Kd", [(10000, 3072, 768), (12000, 768, 768), (5000, 768, 768), (2000, 768, 192),
                                    (333, 520, 256)])
def test_gemm_dropout_masks_every_tile(K, M, N, Kd):
    """The dropout keep flags of the fused GEMM epilogues — computed inside the k-loop on the fast
    path (gemm_common.h epi_bits_step, round 6) or hashed in the epilogue (odd counter offset) — equal
    the standalone dropout kernel's mask for the same counters, on every tile height (128 / 96 / 160
    / 192 rows) and for the ReLU, residual and GELU sites.  A bias of 30 keeps every activation
    positive, so the zero pattern of the output is the mask."""
    x = (0.1 * torch.randn(M, Kd, device="cuda")).half()
    W = (0.05 * torch.randn(N, Kd, device="cuda")).half()
    big = torch.full((N,), 30.0, device="cuda").half()
    zero = torch.zeros(M, N, device="cuda").half()
    z = torch.empty(M, N, device="cuda").half()
    try:
        for mode in (0, 2, 3, 5):
            K.call("mms2ut_gemm_set_tall", mode)
            for seed, off in ((77, 4096), (78, 4097), (79, 2 ** 33 - 4 * N)):
                m = K.dropout_mask(M * N, 0.1, seed, off, "cuda").view(M, N) != 0
                for epi, kw in ((K.EPI_RELU_DROP, {}), (K.EPI_DROP_RESID, dict(aux=zero)),
                                (K.EPI_GELU_DROP, dict(out2=z))):
                    y = K.linear(x, W, big, epi=epi, p=0.1, drop=(seed, off), **kw)
                    assert torch.equal(y != 0, m), (mode, seed, off, epi)
    finally:
        K.call("mms2ut_gemm_set_tall", 1)


@pytest.mark.parametrize("rows,lds,ldd,cols,zcols", [(577, 768, 1536, 768, 768), (33, 85, 96, 85, 11),
                                                       (8, 443136, 443904, 443136, 768), (5, 0, 40, 0, 24)])
def test_copy2d_pad(K, rows, lds, ldd, cols, zcols):
    """mms2ut_copy2d_pad: rows copied and the pad columns zeroed in one launch (vector and scalar
    forms; src NULL = strided zero fill), nothing else in dst touched."""
    src = torch.randn(max(rows * lds, 1), device="cuda").half()
    dst = torch.full((rows * ldd + 16,), 7.0, device="cuda").half()
    ref = dst.clone()
    K.call("mms2ut_copy2d_pad", src.data_ptr() if cols else 0, lds, dst.data_ptr(), ldd, rows, cols, zcols, K._s())
    for r in range(rows):
        ref[r * ldd:r * ldd + cols] = src[r * lds:r * lds + cols]
        ref[r * ldd + cols:r * ldd + cols + zcols] = 0
    torch.cuda.synchronize()
    assert torch.equal(dst, ref)


def test_wgrad_splitk(K):
    M, N, K_ = 5000, 96, 200
    dy = torch.randn(M, N, device="cuda").half()
    x = torch.randn(M, K_, device="cuda").half()
    dW = torch.empty(N, K_, dtype=torch.float16, device="cuda")
    K.linear_wgrad(dy, x, dW)
    torch.cuda.synchronize()
    assert rel(dW, dy.float().t() @ x.float()) < 2e-3


@pytest.mark.parametrize("extra", [True, False])
def test_layernorm_padded_dropout(K, extra):
    """layernorm_fwd_ex / layernorm_bwd_ex (the fusion image path) are bit-identical to the unfused
    LN -> dropout -> copy into the [B, Ti+1, D] key layout, and to the copy-back -> dropout -> LN
    backward (gamma/beta grads)."""
    B, Ti, D, p, drop = 3, 37, 768, 0.1, (11, 8192)
    Tk = Ti + 1 if extra else Ti
    x = (2 * torch.randn(B * Ti, D, device="cuda") + 0.5).half()
    g = (1 + 0.1 * torch.randn(D, device="cuda")).half()
    b = (0.1 * torch.randn(D, device="cuda")).half()
    y0, m0, r0 = K.layernorm(x, g, b)
    ref = torch.zeros(B, Tk, D, dtype=torch.float16, device="cuda")
    ref[:, :Ti] = K.dropout(y0, p, drop).view(B, Ti, D)
    out = torch.full((B, Tk, D), 7.0, dtype=torch.float16, device="cuda")
    if extra:
        out[:, Ti:].zero_()
    _, m1, r1 = K.layernorm(x, g, b, out=out, grp=Ti if extra else 0, grp_out=Tk if extra else 0, p=p,
                            drop=drop)
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and torch.equal(m0, m1) and torch.equal(r0, r1)
    dyp = torch.randn(B * Tk, D, device="cuda").half()
    dy = K.dropout(dyp.view(B, Tk, D)[:, :Ti].clone().view(B * Ti, D), p, drop)
    dgb0, dgb1 = (torch.empty(2 * D, dtype=torch.float16, device="cuda") for _ in range(2))
    K.layernorm_bwd(dy, x, g, m0, r0, dgb0, want_dx=False)
    K.layernorm_bwd(dyp, x, g, m0, r0, dgb1, want_dx=False, dy_grp=Ti if extra else 0,
                    dy_grp_out=Tk if extra else 0, dy_p=p, dy_drop=drop)
    torch.cuda.synchronize()
    assert torch.equal(dgb0, dgb1)


def test_layernorm_fwd_bwd(K):
    """D % 256 == 0 takes the 16-B half-wave-per-row kernels, D = 96 the one-wave-per-row ones."""
    # 46160 rows (the image LayerNorm of a 80-utterance ViT batch): each 16-B-path block folds
    # several 8-row groups into one dgamma / dbeta partial row (ops.hip ln16_iters)
    for R, D in ((1000, 768), (37, 256), (5, 96), (3, 1024), (46160, 768)):
        x = (3 * torch.randn(R, D, device="cuda") + 1).half()
        g = (1 + 0.1 * torch.randn(D, device="cuda")).half()
        b = (0.1 * torch.randn(D, device="cuda")).half()
        y, mean, rstd = K.layernorm(x, g, b)
        xf = x.float().requires_grad_(True)
        gf, bf = g.float().requires_grad_(True), b.float().requires_grad_(True)
        yr = torch.nn.functional.layer_norm(xf, (D,), gf, bf, 1e-5)
        assert rel(y, yr) < 2e-3
        dy = torch.randn(R, D, device="cuda").half()
        dres = torch.randn(R, D, device="cuda").half()
        dgb = torch.empty(2 * D, dtype=torch.float16, device="cuda")
        dx = K.layernorm_bwd(dy, x, g, mean, rstd, dgb, dres=dres)
        yr.backward(dy.float())
        torch.cuda.synchronize()
        assert rel(dx, xf.grad + dres.float()) < 3e-3
        assert rel(dgb[:D], gf.grad) < 3e-3
        assert rel(dgb[D:], bf.grad) < 3e-3
        # fused residual-branch dropout of the gradient: dxd == dropout(dx) with the site's counters
        dx2, dxd = K.layernorm_bwd(dy, x, g, mean, rstd, dgb, dres=dres, emit=(0.1, (7, 4096)))
        keep = K.dropout_mask(R * D, 0.1, 7, 4096, x.device).view(R, D).bool()
        torch.cuda.synchronize()
        assert torch.equal(dx2, dx)
        ref = torch.where(keep, dx.float() / 0.9, torch.zeros_like(dx.float()))
        assert (dxd.float() - ref).abs().max().item() <= 2e-3 * ref.abs().max().item() + 1e-3
        # zero exactly where dropped or dx == 0 — up to elements at the fp16 underflow edge, where the
        # fp32 value behind dx rounds to 0 but its /(1-p) copy does not (or vice versa)
        mism = (dxd == 0) != (~keep | (dx == 0))
        assert (dx.float().abs()[mism] < 1e-6).all() and (dxd.float().abs()[mism] < 1e-6).all()
        # parameter-grad-only mode (image LN: no dx)
        dgb2 = torch.empty_like(dgb)
        assert K.layernorm_bwd(dy, x, g, mean, rstd, dgb2, want_dx=False) is None
        torch.cuda.synchronize()
        assert torch.equal(dgb2, dgb)


@pytest.mark.parametrize("causal,extra", [(False, False), (True, False), (False, True)])
def test_attn_softmax(K, causal, extra):
    Bt, H, Tq, Tk = 3, 2, 19, 23 if not causal else 19
    if extra:
        Tk += 1
    ldS = (Tk + 7) // 8 * 8
    S = torch.randn(Bt * H * Tq * ldS, device="cuda").half()
    lens = torch.tensor([Tk - (1 if extra else 0), 11, 5], dtype=torch.int32, device="cuda")
    P, Pd = K.attn_softmax(S, Bt * H, H, Tq, Tk, ldS, key_len=lens, causal=causal, extra_key=extra)
    s = S.view(Bt, H, Tq, ldS)[..., :Tk].float()
    j = torch.arange(Tk, device="cuda")
    mask = j[None, None, None, :] >= lens.long()[:, None, None, None]
    if extra:
        mask = mask & (j != Tk - 1)
    if causal:
        mask = mask | (j[None, None, None, :] > torch.arange(Tq, device="cuda")[None, None, :, None])
    sf = s.masked_fill(mask, float("-inf")).requires_grad_(True)
    pr = torch.softmax(sf, -1)
    assert rel(P.view(Bt, H, Tq, ldS)[..., :Tk], pr) < 2e-3
    dP = torch.randn(Bt * H * Tq * ldS, device="cuda").half()
    pr.backward(dP.view(Bt, H, Tq, ldS)[..., :Tk].float())
    dS = K.attn_softmax_bwd(P, dP.clone(), Bt * H, H, Tq, Tk, ldS)
    torch.cuda.synchronize()
    assert rel(dS.view(Bt, H, Tq, ldS)[..., :Tk], sf.grad.nan_to_num(0.0)) < 3e-3


@pytest.mark.parametrize("Tk", [101, 578, 1031])
@pytest.mark.parametrize("masked", [False, True])
def test_attn_softmax_fusion_widths(K, Tk, masked):
    """The fusion attention's widths: DETR 100 + bias_kv (101), ViT 577 + bias_kv (578, the
    3-chunks-per-lane instantiation) and one past it, with image key masks, the extra bias_kv key
    and attention dropout 0.1 replayed from the HIP RNG."""
    Z, Tq, p = 5, 37, 0.1
    ldS = (Tk + 7) // 8 * 8
    g = torch.Generator(device="cuda").manual_seed(Tk)
    S = (3 * torch.randn(Z * Tq * ldS, device="cuda", generator=g)).half()
    km = None
    if masked:
        km = torch.zeros(Z, ldS, dtype=torch.uint8, device="cuda")
        for z in range(Z):
            km[z, max(1, (Tk - 1) * (z + 1) // (Z + 1)):Tk - 1] = 1   # padded image keys; bias_kv column kept
    P, Pd = K.attn_softmax(S, Z, 1, Tq, Tk, ldS, key_mask=km, extra_key=True, p=p, drop=(11, 512))
    s = S.view(Z, Tq, ldS)[..., :Tk].float()
    if km is not None:
        s = s.masked_fill(km[:, None, :Tk].bool(), float("-inf"))
    sf = s.clone().requires_grad_(True)
    pr = torch.softmax(sf, -1)
    m = K.dropout_mask(Z * Tq * Tk, p, 11, 512, "cuda").view(Z, Tq, Tk).float()
    assert rel(P.view(Z, Tq, ldS)[..., :Tk], pr) < 2e-3
    assert rel(Pd.view(Z, Tq, ldS)[..., :Tk], pr * m / (1 - p)) < 2e-3
    dPd = torch.randn(Z * Tq * ldS, device="cuda", generator=g).half()
    (pr * m / (1 - p)).backward(dPd.view(Z, Tq, ldS)[..., :Tk].float())
    dS = K.attn_softmax_bwd(P, dPd.clone(), Z, 1, Tq, Tk, ldS, p=p, drop=(11, 512))
    torch.cuda.synchronize()
    assert rel(dS.view(Z, Tq, ldS)[..., :Tk], sf.grad.nan_to_num(0.0)) < 3e-3


def test_attn_softmax_dropout_replay(K):
    Z, Tq, Tk = 4, 16, 30
    ldS = 32
    S = torch.randn(Z * Tq * ldS, device="cuda").half()
    P, Pd = K.attn_softmax(S, Z, 1, Tq, Tk, ldS, p=0.2, drop=(7, 0))
    m = K.dropout_mask(Z * Tq * Tk, 0.2, 7, 0, "cuda").view(Z, Tq, Tk).float()
    pv = P.view(Z, Tq, ldS)[..., :Tk].float()
    torch.cuda.synchronize()
    assert rel(Pd.view(Z, Tq, ldS)[..., :Tk], pv * m / 0.8) < 2e-3
    # backward with the same mask
    pf = torch.softmax(S.view(Z, Tq, ldS)[..., :Tk].float(), -1).requires_grad_(True)
    out = pf * m / 0.8
    g = torch.randn(Z * Tq * ldS, device="cuda").half()
    out.backward(g.view(Z, Tq, ldS)[..., :Tk].float())
    # d(softmax) from d(pf)
    pr = torch.softmax(S.view(Z, Tq, ldS)[..., :Tk].float(), -1)
    dS_ref = pr * (pf.grad - (pf.grad * pr).sum(-1, keepdim=True))
    dS = K.attn_softmax_bwd(P, g.clone(), Z, 1, Tq, Tk, ldS, p=0.2, drop=(7, 0))
    torch.cuda.synchronize()
    assert rel(dS.view(Z, Tq, ldS)[..., :Tk], dS_ref) < 3e-3


def _attn_ref(q, k, v, lens, causal, scale, mask=None):
    s = scale * q @ k.transpose(-1, -2)
    Tq, Tk = s.shape[-2], s.shape[-1]
    j = torch.arange(Tk, device=s.device)
    bad = j[None, None, None, :] >= lens.long()[:, None, None, None]
    if causal:
        bad = bad | (j[None, None, None, :] > torch.arange(Tq, device=s.device)[None, None, :, None])
    p = torch.softmax(s.masked_fill(bad, float("-inf")), -1)
    if mask is not None:
        p = p * mask
    return p @ v


_FLASH_CASES = [
    (False, 70, 90, [90, 50, 7], 0.0), (True, 70, 70, [70, 41, 3], 0.0),
    (False, 130, 130, [130, 129, 65], 0.0), (True, 150, 150, [150, 100, 1], 0.25),
    (False, 33, 200, [200, 64, 63], 0.1), (True, 128, 128, [128, 77, 5], 0.1),
    (False, 100, 128, [128, 100, 1], 0.2), (False, 1, 17, [17, 9, 1], 0.0),
    (False, 300, 100, [100, 57, 2], 0.1), (True, 256, 256, [256, 200, 9], 0.1),
    (False, 301, 213, [213, 129, 1], 0.1), (True, 257, 257, [257, 130, 4], 0.0),
    (False, 70, 300, [300, 257, 3], 0.1), (True, 300, 300, [300, 129, 2], 0.2)]
# the many-heads variant only where it targets the fused kernel (Tq <= 130, Tk <= 256)
_FLASH_PARAMS = [c + ("few",) for c in _FLASH_CASES] + \
    [c + ("many",) for c in _FLASH_CASES if c[1] <= 130 and c[2] <= 256]


@pytest.mark.parametrize("hd", [64, 96])
@pytest.mark.parametrize("causal,Tq,Tk,lens,p,heads", _FLASH_PARAMS)
def test_flash_attention_fwd_bwd(K, hd, causal, Tq, Tk, lens, p, heads):
    """Tk <= 256 takes the one-launch chunked backward (any Tq), Tk > 256 the three-kernel one.
    heads=many: B*H = 3*96 = 288 heads > 256 CUs, so persistent blocks of the fused kernel walk
    several heads (the next-head prefetch path)."""
    B, H = 3, (2 if heads == "few" else 96)
    d = H * hd
    g = torch.Generator(device="cuda").manual_seed(5)
    q = torch.randn(B * Tq, d, generator=g, device="cuda").half()
    kv = torch.randn(B * Tk, 2 * d, generator=g, device="cuda").half()
    lens_t = torch.tensor(lens, dtype=torch.int32, device="cuda")
    o = torch.empty(B * Tq, d, dtype=torch.float16, device="cuda")
    seed, off = 77, 1024
    lse = K.mha_fwd(q, kv, kv[:, d:], o, d, 2 * d, 2 * d, d, B, H, Tq, Tk, hd, hd ** -0.5, key_len=lens_t,
                    causal=causal, p=p, drop=(seed, off))
    qf = q.float().view(B, Tq, H, hd).transpose(1, 2).requires_grad_(True)
    kf = kv[:, :d].float().view(B, Tk, H, hd).transpose(1, 2).requires_grad_(True)
    vf = kv[:, d:].float().view(B, Tk, H, hd).transpose(1, 2).requires_grad_(True)
    mask = None
    if p > 0:
        mask = K.dropout_mask(B * H * Tq * Tk, p, seed, off, "cuda").view(B, H, Tq, Tk).float() / (1 - p)
    ref = _attn_ref(qf, kf, vf, lens_t, causal, hd ** -0.5, mask)
    got = o.float().view(B, Tq, H, hd).transpose(1, 2)
    torch.cuda.synchronize()
    assert rel(got, ref) < 3e-3
    do = torch.randn(B * Tq, d, generator=g, device="cuda").half()
    ref.backward(do.float().view(B, Tq, H, hd).transpose(1, 2))
    dq = torch.empty_like(q)
    dkv = torch.empty_like(kv)
    K.mha_bwd(q, kv, kv[:, d:], o, d, 2 * d, 2 * d, d, B, H, Tq, Tk, hd, hd ** -0.5, lens_t, causal, p,
              (seed, off), lse, do, d, dq, d, dkv, 2 * d, dkv[:, d:], 2 * d)
    torch.cuda.synchronize()
    t = lambda x, T: x.float().view(B, T, H, hd).transpose(1, 2)
    assert rel(t(dq, Tq), qf.grad) < 5e-3
    # keys beyond the length get exactly zero gradient (as the reference's masked softmax)
    assert rel(t(dkv[:, :d], Tk), kf.grad) < 5e-3
    assert rel(t(dkv[:, d:], Tk), vf.grad) < 5e-3


def test_ls_xent(K):
    rows, V, eps, pad = 333, 1004, 0.2, 1
    Vp = 1008
    logits = torch.randn(rows, Vp, device="cuda").half()
    target = torch.randint(0, V, (rows,), device="cuda")
    target[::7] = pad
    out = torch.zeros(2, device="cuda")
    lse = K.ls_xent_fwd(logits, Vp, target, rows, V, eps, pad, out)
    z = logits[:, :V].float().requires_grad_(True)
    lp = torch.log_softmax(z, -1)
    keep = target != pad
    nll = -lp[keep, target[keep]].sum()
    smooth = -lp[keep].sum()
    ei = eps / (V - 1)
    loss = (1 - eps - ei) * nll + ei * smooth
    torch.cuda.synchronize()
    assert abs(out[0].item() - loss.item()) / loss.item() < 1e-4
    assert abs(out[1].item() - nll.item()) / nll.item() < 1e-4
    loss.backward()
    g = torch.tensor([3.0], device="cuda")
    dz = torch.empty_like(logits)
    dz.fill_(float("nan"))
    K.ls_xent_bwd(logits, Vp, target, rows, V, eps, pad, lse, g, dz)
    torch.cuda.synchronize()
    assert rel(dz[:, :V], 3 * z.grad) < 2e-3
    assert torch.equal(dz[:, V:], torch.zeros_like(dz[:, V:]))  # pad columns zeroed


@pytest.mark.parametrize("B,Tin,C,k,ldcol", [(3, 41, 80, 5, 448), (2, 37, 512, 5, None), (2, 23, 6, 5, None),
                                             (4, 250, 80, 5, 400)])
def test_im2col_col2im_exact(K, B, Tin, C, k, ldcol):
    """im2col is a pure gather: bit-exact against torch unfold (zero pad columns past C*k); col2im
    sums <= ceil(k/stride) taps in fp32: against the fp32 fold, one fp16 rounding apart.  Covers the
    vectorised kernels (ldcol % 8 == 0, C % 4 == 0) and the generic ones (C = 6, ldcol = 30)."""
    Tout = (Tin - 1) // 2 + 1
    x = torch.randn(B * Tin, C, device="cuda").half()
    col = K.im2col(x, B, Tin, Tout, C, k, ldcol=ldcol)
    ref = torch.nn.functional.unfold(x.view(B, Tin, C).transpose(1, 2).unsqueeze(-1).float(), (k, 1),
                                     padding=(2, 0), stride=(2, 1)).transpose(1, 2).reshape(B * Tout, C * k)
    W = C * k
    assert torch.equal(col[:, :W].float(), ref)
    if col.shape[1] > W:
        assert torch.equal(col[:, W:], torch.zeros_like(col[:, W:]))
    dcol = torch.randn(B * Tout, W, device="cuda").half()
    dx = K.col2im(dcol, B, Tin, Tout, C, k)
    fold = torch.nn.functional.fold(dcol.float().view(B, Tout, W).transpose(1, 2), (Tin, 1), (k, 1),
                                    padding=(2, 0), stride=(2, 1)).view(B, C, Tin).transpose(1, 2).reshape(B * Tin, C)
    assert torch.equal(dx, fold.half())


def test_glu_im2col_col2im(K):
    B, Tin, C, k = 2, 23, 16, 5
    Tout = (Tin - 1) // 2 + 1
    x = torch.randn(B * Tin, C, device="cuda").half()
    col = K.im2col(x, B, Tin, Tout, C, k)
    W = torch.randn(8, C, k, device="cuda")
    ref = torch.nn.functional.conv1d(x.float().view(B, Tin, C).transpose(1, 2), W, stride=2, padding=2)
    got = (col.float() @ W.view(8, -1).t()).view(B, Tout, 8).transpose(1, 2)
    assert rel(got, ref) < 2e-3
    dcol = torch.randn_like(col)
    dx = K.col2im(dcol, B, Tin, Tout, C, k)
    xf = x.float().requires_grad_(True)
    col_ref = torch.nn.functional.unfold(xf.view(B, Tin, C).transpose(1, 2).unsqueeze(-1), (k, 1),
                                         padding=(2, 0), stride=(2, 1))  # [B, C*k, Tout]
    col_ref.backward(dcol.float().view(B, Tout, C * k).transpose(1, 2))
    torch.cuda.synchronize()
    assert rel(dx, xf.grad) < 2e-3
    h = torch.randn(50, 64, device="cuda").half()
    y = K.glu(h, 32)
    hf = h.float().requires_grad_(True)
    yr = torch.nn.functional.glu(hf, -1)
    assert rel(y, yr) < 2e-3
    dy = torch.randn(50, 32, device="cuda").half()
    dh = K.glu_bwd(h, dy, 32)
    yr.backward(dy.float())
    torch.cuda.synchronize()
    assert rel(dh, hf.grad) < 3e-3


@pytest.mark.parametrize("rows", [9000, 777, 1, 0])
def test_wgrad_group(K, rows):
    """One grouped launch == each product in fp32 (encoder-layer shapes, ragged N / K multiples of
    8, one problem without a bias, strided dy / x views as the layer scratch holds them); rows = 0
    writes zeros.  Deterministic: a second launch is bit-identical."""
    g = torch.Generator(device="cuda").manual_seed(rows)
    shapes = [(2304, 768, True), (768, 768, True), (3072, 768, True), (768, 3072, True), (200, 136, False)]
    probs = []
    for N, K_, bias in shapes:
        dyb = (torch.randn(rows, N + 8, device="cuda", generator=g) * 0.1).half()
        xb = torch.randn(rows, K_ + 16, device="cuda", generator=g).half()
        dW = torch.full((N, K_), 7.0, dtype=torch.float16, device="cuda")
        db = torch.full((N,), 7.0, dtype=torch.float16, device="cuda") if bias else None
        probs.append((dyb[:, :N], xb[:, :K_], dW, db))
    K.wgrad_group(probs, rows)
    first = [p[2].clone() for p in probs]
    K.wgrad_group(probs, rows)
    torch.cuda.synchronize()
    for (dy, x, dW, db), f in zip(probs, first):
        assert torch.equal(dW, f)
        ref = dy.float().t() @ x.float()
        if rows == 0:
            assert not dW.any() and (db is None or not db.any())
            continue
        assert rel(dW, ref) < 2e-3
        if db is not None:
            assert rel(db, dy.float().sum(0)) < 2e-3


@pytest.mark.parametrize("M,N,K_", [(5000, 96, 256), (8704, 768, 768), (1000, 200, 64), (77, 2304, 128)])
def test_wgrad_fused_bias(K, M, N, K_):
    """dW and db from one GEMM launch (db = the A-row sums of the first tile column)."""
    dy = torch.randn(M, N, device="cuda").half()
    x = torch.randn(M, K_, device="cuda").half()
    dW = torch.empty(N, K_, dtype=torch.float16, device="cuda")
    db = torch.full((N,), 7.0, dtype=torch.float16, device="cuda")
    K.linear_wgrad(dy, x, dW, db=db, side=False)
    torch.cuda.synchronize()
    assert rel(dW, dy.float().t() @ x.float()) < 2e-3
    assert rel(db, dy.float().sum(0)) < 2e-3


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K_", [(4100, 1540, 2048), (4233, 1600, 2112)])
def test_gemm_tile256(K, a_kc, b_kc, M, N, K_):
    """The 256x256-tile ring kernel (taken for M >= 4096, N >= 1536, K >= 2048) on ragged shapes and
    every operand layout."""
    A = _mat(M, K_, seed=1) if a_kc else _mat(K_, M, ld=(M + 7) // 8 * 8, seed=1)
    B = _mat(N, K_, seed=2) if b_kc else _mat(K_, N, ld=(N + 7) // 8 * 8, seed=2)
    Af = A.float() if a_kc else A.float().t()
    Bf = B.float() if b_kc else B.float().t()
    ldc = (N + 7) // 8 * 8
    C = torch.zeros(M, ldc, dtype=torch.float16, device="cuda")
    K.gemm(A, B, C, M, N, K_, a_kc=a_kc, b_kc=b_kc, lda=A.stride(0), ldb=B.stride(0), ldc=ldc)
    torch.cuda.synchronize()
    assert rel(C[:, :N], Af @ Bf.t()) < 2e-3


def test_transposed_weight_images_many(K):
    """More descriptors than one wave's lanes (the block's matrix lookup counts them 256 at a time):
    300 ragged matrices, every image equals W^T."""
    g = torch.Generator().manual_seed(5)
    shapes = [(8 * int(torch.randint(1, 20, (1,), generator=g)), 8 * int(torch.randint(1, 20, (1,), generator=g)))
              for _ in range(300)]
    flat = torch.randn(sum(r * c for r, c in shapes) + 8 * len(shapes), device="cuda").half()
    mats, off = [], 0
    for r, c in shapes:
        mats.append(flat[off:off + r * c].view(r, c))
        off += r * c + 8
    wt = K.TransposedWeights(flat, mats)
    wt.refresh()
    for W in mats:
        T = wt.get(W)
        torch.cuda.synchronize()
        assert T is not None and torch.equal(T, W.t())


def test_transposed_weight_images(K):
    """One transpose_batch launch writes W^T for every registered matrix (ragged tile edges); the
    dgrad through the image equals the dgrad through W."""
    flat = torch.randn(200_000, device="cuda").half()
    mats = [flat[:72 * 136].view(72, 136), flat[10_000:10_000 + 256 * 64].view(256, 64),
            flat[40_000:40_000 + 200 * 96].view(200, 96)]
    wt = K.TransposedWeights(flat, mats)
    wt.refresh()
    for W in mats:
        T = wt.get(W)
        torch.cuda.synchronize()
        assert T is not None and torch.equal(T, W.t())
    dy = torch.randn(333, 200, device="cuda").half()
    ref = K.linear_dgrad(dy, mats[2])
    K.TransposedWeights.active = wt
    try:
        got = K.linear_dgrad(dy, mats[2])
    finally:
        K.TransposedWeights.active = None
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("B,T,D,V,p", [(37, 301, 768, 1004, 0.1), (3, 50, 256, 40, 0.0), (1, 1, 512, 7, 0.3),
                                       (64, 200, 1024, 1004, 0.1)])
def test_token_embed_bwd(K, B, T, D, V, p):
    """Embedding-gradient scatter (csrc/ops.hip token_embed_bwd_kernel) against torch index_add of the
    scaled, dropout-masked rows (mask from the library's own counter RNG); the pad row gets nothing;
    run twice into the same accumulator: bit-identical increments (deterministic order)."""
    g = torch.Generator(device="cuda").manual_seed(7)
    pad = 1
    tok = torch.randint(0, V, (B, T), generator=g, device="cuda")
    tok[:, -T // 5:] = pad
    dx = torch.randn(B * T, D, generator=g, device="cuda").half()
    scale, seed, off = math.sqrt(D), 123, 4096
    dE = torch.zeros(V, D, device="cuda")
    K.token_embed_bwd(tok, dx, dE, B, T, D, pad, scale, p, (seed, off))
    first = dE.clone()
    K.token_embed_bwd(tok, dx, dE, B, T, D, pad, scale, p, (seed, off))
    torch.cuda.synchronize()
    x = dx.float() * scale
    if p > 0:
        keep = K.dropout_mask(B * T * D, p, seed, off, "cuda").view(B * T, D).bool()
        x = torch.where(keep, x / (1 - p), torch.zeros_like(x))
    ref = torch.zeros(V, D, device="cuda").index_add_(0, tok.reshape(-1), x)
    ref[pad] = 0
    assert rel(first, ref) < 1e-5
    assert torch.equal(first[pad], torch.zeros_like(first[pad]))
    assert torch.equal(dE, first + first)
