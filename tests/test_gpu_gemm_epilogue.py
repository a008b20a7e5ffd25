"""The register epilogue (csrc/gemm_common.h reg_epilogue: plain / bias and ReLU-dropout element math on
the accumulators in the MFMA layout, fp16 staged through LDS) against the fp32-staged epilogue it
replaces (mms2ut_gemm_set_epilogue(1)), bit for bit, over every kernel that carries it: the tall NT
tiles (96 / 160 / 192 rows), the 128x128 LDS-DMA and register-staged kernels, the 256x256 kernel, the
batched attention products (alpha != 1) and the grouped weight gradients.  Also the launch-uniform
path choice: N = 1004 (the unit vocabulary, padded ldc 1024) takes the staged path in every wave —
a per-wave choice there mixed the two LDS slot layouts inside one block (round 6), which only a
repeated run exposes, so every case runs several times; N = 320 / 192 leave a block's second
64-column half past N (that wave returns early).  Dropout streams as the step uses them: large
and odd counter offsets, seeds per site."""
import pytest
import torch

from conftest import pkg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K_():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg().kernels


def _both(K_, fn, reps=3):
    """fn() under the register epilogue (reps times, all equal) and under the staged one."""
    outs = []
    try:
        for staged in (0, 1):
            K_.call("mms2ut_gemm_set_epilogue", staged)
            for _ in range(reps if staged == 0 else 1):
                outs.append(fn().clone())
    finally:
        K_.call("mms2ut_gemm_set_epilogue", 0)
    torch.cuda.synchronize()
    ref = outs[-1].view(torch.int16)
    for i, o in enumerate(outs[:-1]):
        assert torch.equal(o.view(torch.int16), ref), f"run {i}: {(o.view(torch.int16) != ref).sum().item()} bits differ"
    return outs[-1]


@pytest.mark.parametrize("M,N,Kd", [(9607, 3072, 768), (11003, 768, 768), (7589, 2304, 768), (12000, 768, 3072),
                                    (2000, 768, 768), (3011, 1004, 768), (777, 3072, 768), (131, 768, 768),
                                    (1500, 320, 768), (9, 192, 256)])
def test_linear_epilogues_bit_identical(K_, M, N, Kd):
    g = torch.Generator(device="cuda").manual_seed(M + N + Kd)
    x = (torch.randn(M, Kd, device="cuda", generator=g) * 0.5).half()
    W = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).half()
    b = (torch.randn(N, device="cuda", generator=g) * 0.1).half()
    _both(K_, lambda: K_.linear(x, W))
    _both(K_, lambda: K_.linear(x, W, b))
    for seed, off in ((1234, 0), (77, 7), (5, (1 << 33) - 12345678), (9, 123456789012)):
        _both(K_, lambda: K_.linear(x, W, b, epi=K_.EPI_RELU_DROP, p=0.1, drop=(seed, off)))
    big = (x * 60).half()   # accumulators past the fp16 range: inf / relu(inf) paths
    _both(K_, lambda: K_.linear(big, W * 40, b, epi=K_.EPI_RELU_DROP, p=0.1, drop=(3, 64)))
    if N == 1004:   # the logits GEMM: N = 1004 inside a 1024-column row
        out = torch.zeros(M, 1024, dtype=torch.float16, device="cuda")

        def logits():
            K_.gemm(x, W, out, M, N, Kd, lda=Kd, ldb=Kd, ldc=1024)
            return out
        _both(K_, logits, reps=5)


def test_batched_alpha_bit_identical(K_):
    """Attention-shaped batched products with alpha = 1/sqrt(hd) (QK^T: A, B K-contiguous; PV: B
    N-contiguous)."""
    g = torch.Generator(device="cuda").manual_seed(3)
    Bh, T, S, hd = 24, 250, 577, 64
    q = torch.randn(Bh, T, hd, device="cuda", generator=g).half()
    k = torch.randn(Bh, S, hd, device="cuda", generator=g).half()
    v = torch.randn(Bh, S, 128, device="cuda", generator=g).half()
    sc = torch.empty(Bh, T, 640, dtype=torch.float16, device="cuda")
    o = torch.empty(Bh, T, 128, dtype=torch.float16, device="cuda")

    def qk():
        K_.gemm(q, k, sc, T, S, hd, lda=hd, ldb=hd, ldc=640, batch=Bh, sA=(T * hd, 0), sB=(S * hd, 0),
                sC=(T * 640, 0), alpha=hd ** -0.5)
        return sc[:, :, :S]

    def pv():
        K_.gemm(sc, v, o, T, 128, 576, lda=640, ldb=128, ldc=128, b_kc=False, batch=Bh, sA=(T * 640, 0),
                sB=(S * 128, 0), sC=(T * 128, 0), alpha=0.5)
        return o
    _both(K_, qk)
    _both(K_, pv)


def test_wgrad_group_bit_identical(K_):
    g = torch.Generator(device="cuda").manual_seed(11)
    rows = 9607
    probs = []
    for N, Kin, bias in [(2304, 768, True), (768, 768, True), (3072, 768, True), (768, 3072, True), (200, 136, False)]:
        dy = (torch.randn(rows, N, device="cuda", generator=g) * 0.1).half()
        x = torch.randn(rows, Kin, device="cuda", generator=g).half()
        probs.append((dy, x, torch.empty(N, Kin, dtype=torch.float16, device="cuda"),
                      torch.empty(N, dtype=torch.float16, device="cuda") if bias else None))

    def run():
        K_.wgrad_group(probs, rows)
        return torch.cat([p[2].flatten() for p in probs] + [p[3] for p in probs if p[3] is not None])
    _both(K_, run)
