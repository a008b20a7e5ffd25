"""Torch-tensor front of the C-ABI: validation + pointer plumbing, no arithmetic.

Every function enqueues HIP kernels on PyTorch's current stream through libmms2ut_hip.so.
Tensors are fp16 (``torch.float16``) unless stated; shapes are checked before the call.
"""
import atexit
import ctypes
import math
import os

import torch

from . import _lib
from ._lib import GemmArgs, call

EPI_F16, EPI_RELU_DROP, EPI_DROP_RESID, EPI_F32, EPI_GATE, EPI_RELU_DROP_BWD, EPI_F16_ACC, EPI_GELU_DROP, \
    EPI_GELU_DROP_BWD = range(9)
F16 = torch.float16


_DEV = [None]


def _dev():
    if _DEV[0] is None:
        _DEV[0] = torch.cuda.current_device()
    return _DEV[0]


def _s():
    """Raw hipStream_t to enqueue on: the side stream inside a side region, else torch's current
    stream (read through the C binding: torch.cuda.current_stream() costs ~5 us per call)."""
    return _Side.override or torch._C._cuda_getCurrentRawStream(_dev())


def _p(t):
    return None if t is None else t.data_ptr()


def _chk(t, dtype=F16):
    assert t.is_cuda, "HIP kernels need device tensors"
    assert t.dtype == dtype, f"expected {dtype}, got {t.dtype}"


class Dropout:
    """Counter-based dropout stream: each call site draws a disjoint counter range from one
    per-step seed, so a backward pass regenerates exactly the forward mask."""

    def __init__(self, seed=1):
        self.seed = seed
        self.offset = 0

    def reset(self, seed):
        self.seed = int(seed) & ((1 << 63) - 1)
        self.offset = 0

    def take(self, n):
        off = self.offset
        self.offset += (int(n) + 255) // 256 * 256
        return self.seed, off

# ============================================================================ GEMM


def gemm(A, B, C, M, N, K, *, a_kc=True, b_kc=True, lda, ldb, ldc, batch=1, bdiv=1,
         sA=(0, 0), sB=(0, 0), sC=(0, 0), epi=EPI_F16, alpha=1.0, bias=None, aux=None, ldaux=0,
         sX=(0, 0), out2=None, ldo2=0, p=0.0, seed=0, offset=0, ld_rng=0, splitk=1, sCsplit=0,
         rowsum=None, ld_rowsum=0, fixup=True):
    """One mms2ut_gemm_f16 launch.  The argument block is packed in one struct call (_lib.GEMM_ARGS,
    the C layout of mms2ut_gemm_args).  Short-M fused-epilogue GEMMs take the split-K fixup
    (fixup=False: the unsplit kernel, for tests)."""
    ws_p = ws_n = 0
    if fixup and splitk == 1 and epi != EPI_F32 and batch == 1 and rowsum is None:
        s = _fixup_splits(M, N, K)
        if s > 1:
            ws = _workspace("splitk_fix", s * M * N, C.device)
            splitk, ws_p, ws_n = s, ws.data_ptr(), ws.numel()
    buf = _GEMM_PACK(
        A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, a_kc, b_kc, lda, ldb, ldc, batch, bdiv,
        sA[0], sA[1], sB[0], sB[1], sC[0], sC[1], splitk, sCsplit, epi, alpha,
        0 if bias is None else bias.data_ptr(), 0 if aux is None else aux.data_ptr(), ldaux, sX[0], sX[1],
        0 if out2 is None else out2.data_ptr(), ldo2, p, seed, offset, ld_rng,
        0 if rowsum is None else rowsum.data_ptr(), ld_rowsum, ws_p, ws_n)
    call("mms2ut_gemm_f16", buf, _s())


_GEMM_PACK = _lib.GEMM_ARGS.pack


def _fixup_splits(M, N, K):
    """Split count for a short-M fused-epilogue GEMM (decoder tokens): its 128x128 grid covers a
    fraction of the 256 CUs, so K is split until ~512 workgroups (2 per CU) run, each split keeping
    >= 4 k-tiles (include/mms2ut.h splitk_ws)."""
    if N % 4 or K < 512:
        return 1
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    if tiles >= 128:
        return 1
    return max(1, min(512 // tiles, K // 256, 16))


def gemm_profile_begin(max_launches=100000):
    """Start live GEMM timing (HIP events inside the library, on each launch's stream)."""
    call("mms2ut_profile_begin", int(max_launches))


def gemm_profile_end():
    """-> (summed GEMM kernel ms, launches, launched FLOPs, algorithmic HBM bytes)."""
    import ctypes
    ms, n, fl, by = ctypes.c_float(), ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
    call("mms2ut_profile_end", ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl))
    call("mms2ut_profile_bytes", ctypes.byref(by))
    return ms.value, n.value, fl.value, by.value


def gemm_profile_launches(n):
    """Per-launch (ms, launched FLOPs, class word) of the last gemm_profile window (numpy)."""
    import numpy as np
    ms, fl, cls = np.zeros(n, np.float32), np.zeros(n, np.float64), np.zeros(n, np.int32)
    if n:
        call("mms2ut_profile_launches", ms.ctypes.data, fl.ctypes.data, cls.ctypes.data, int(n))
    return ms, fl, cls


def gemm_profile_shapes(n):
    """[n, 4] int32 (M, N, K, batch * splitk) of the last gemm_profile window's launches."""
    import numpy as np
    mnk = np.zeros((max(n, 0), 4), np.int32)
    if n:
        call("mms2ut_profile_shapes", mnk.ctypes.data, int(n))
    return mnk


def gemm_profile_stamps(buf):
    """Stamp mode for the open profile window: every GEMM kernel's blocks record {start, end}
    s_memrealtime ticks into `buf` (int64 device tensor, 2 per block) instead of HIP events."""
    assert buf.dtype == torch.int64 and buf.is_cuda and buf.numel() % 2 == 0
    call("mms2ut_profile_stamps", buf.data_ptr(), buf.numel() // 2)


def gemm_profile_durations(buf, n):
    """Per-launch kernel durations (ms, numpy float64) of the last stamp-mode window: max(end) -
    min(start) over each launch's blocks; NaN for launches past the buffer's capacity."""
    import ctypes
    import numpy as np
    fl = np.zeros((max(n, 0), 2), np.int64)
    if n:
        call("mms2ut_profile_blocks", fl.ctypes.data, int(n))
    khz = ctypes.c_int()
    call("mms2ut_wallclock_khz", ctypes.byref(khz))
    st = buf.view(-1, 2).cpu().numpy()
    cap = st.shape[0]
    out = np.full(n, np.nan)
    for i, (b0, b1) in enumerate(fl.tolist()):
        if b1 <= cap and b1 > b0:
            out[i] = (st[b0:b1, 1].max() - st[b0:b1, 0].min()) / khz.value   # ticks / kHz = ms
    return out


def linear(x, W, bias=None, out=None, *, epi=EPI_F16, aux=None, out2=None, p=0.0, drop=None,
           ldc=None, alpha=1.0):
    """out[M,N] = epi(x[M,K] @ W[N,K]^T + bias) — nn.Linear forward (fused epilogue)."""
    M, K = x.shape
    N = W.shape[0]
    assert W.shape[1] == K, (W.shape, x.shape)
    if out is None:
        out = torch.empty(M, N, dtype=F16, device=x.device)
    seed = off = 0
    if p > 0.0:
        seed, off = drop
    gemm(x, W, out, M, N, K, lda=x.stride(0), ldb=W.stride(0), ldc=ldc or out.stride(0), epi=epi,
         bias=bias, aux=aux, ldaux=(aux.stride(0) if aux is not None else 0), out2=out2,
         ldo2=(out2.stride(0) if out2 is not None else 0), p=p, seed=seed, offset=off, ld_rng=N,
         alpha=alpha)
    return out


class TransposedWeights:
    """W^T images of the weights the backward's dgrad GEMMs read, in one flat fp16 buffer.

    dx = dy @ W reads W [N, K] N-contiguous (transposed LDS reads); with W^T [K, N] both GEMM
    operands are K-contiguous, the NT layout the forward uses (13-20 % faster on the step's dgrad
    shapes, round-2 A/B, scripts/gemm_ab.py in git history).  refresh() re-transposes every registered matrix in one launch on
    the side stream after each optimizer update (it runs beside the forward); the first dgrad of
    the backward makes the main stream wait for it.  linear_dgrad picks the image up by W's
    address and shape; unregistered weights keep the transposed-read path."""
    active = None

    def __init__(self, flat, mats):
        import numpy as np
        base = flat.data_ptr()
        self.flat = flat
        self.lookup = {}
        rows, off, tiles = [], 0, 0
        for W in mats:
            r, c = W.shape
            assert W.dtype == F16 and W.stride(1) == 1 and W.stride(0) == c and r % 8 == 0 and c % 8 == 0
            src = (W.data_ptr() - base) // 2
            if (src, r, c) in self.lookup:
                continue
            self.lookup[(src, r, c)] = off
            rows.append((src, off, r, c, tiles, 0))
            off = round_up(off + r * c, 8)
            tiles += -(-r // 64) * -(-c // 64)
        dt = np.dtype([("src", "<i8"), ("dst", "<i8"), ("rows", "<i4"), ("cols", "<i4"), ("tile0", "<i4"),
                       ("pad", "<i4")])
        desc = np.array(rows, dtype=dt)
        self.desc = torch.from_numpy(desc.view(np.uint8).copy()).to(flat.device)
        self.n, self.tiles = len(rows), tiles
        self.flatT = torch.empty(max(off, 8), dtype=F16, device=flat.device)
        self.event = None
        self.waited = True

    def refresh(self):
        if self.n == 0:
            return
        side = side_stream(self.flat.device)
        stream_wait(side, torch.cuda.current_stream(self.flat.device))
        with torch.cuda.stream(side):
            call("mms2ut_transpose_batch", self.flat.data_ptr(), self.flatT.data_ptr(), self.desc.data_ptr(),
                 self.n, self.tiles, _s())
        if self.event is None:
            self.event = DevEvent()
        self.event.record(side)
        self.waited = False

    def get(self, W, wait=True):
        if self.event is None or W.dim() != 2:
            return None
        off = self.lookup.get(((W.data_ptr() - self.flat.data_ptr()) // 2, W.shape[0], W.shape[1]))
        if off is None or W.stride(1) != 1 or W.stride(0) != W.shape[1]:
            return None
        if wait:
            self.wait_ready()
        return self.flatT[off:off + W.numel()].view(W.shape[1], W.shape[0])

    def wait_ready(self):
        """The current stream waits for this step's refresh (once per refresh)."""
        if not self.waited and self.event is not None:
            self.event.wait(torch.cuda.current_stream(self.flat.device))
            self.waited = True


_STREAM_WS = {}


def stream_workspace(numel, device):
    """fp32 scratch private to the current stream (grow-only; a regrown buffer is released to the
    caching allocator on the stream that allocated and used it, so later reuse is stream-ordered).
    In graph mode (_Side.retain) a regrown buffer is retired instead: an earlier captured graph
    still writes its split-K partials into it on every replay."""
    if numel <= 0:
        return None
    key = _s()
    buf = _STREAM_WS.get(key)
    if buf is None or buf.numel() < numel:
        if buf is not None and _Side.retain:
            _Side.retired.append(buf)
        buf = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=device)
        _STREAM_WS[key] = buf
    return buf


class LayerCall:
    """One pre-LN transformer layer enqueued by a single library call (include/mms2ut.h
    mms2ut_layer_fwd / mms2ut_layer_bwd: the whole per-layer launch sequence from C++ instead of
    ~25 launches issued one by one from Python).  Parameter, gradient and W^T pointers are bound
    once (the flat buffers never move); each forward sets shapes, lengths, dropout offsets and the
    arena, and snapshots the argument block for its backward."""

    _sizes = {}

    def __init__(self, kind, d, H, F, params, grads, dgrad_weights, eps=1e-5):
        a = _lib.LayerArgs()
        a.kind, a.d, a.H, a.F, a.eps = kind, d, H, F, eps
        for f, t in params.items():
            setattr(a, f, t.data_ptr())
        for f, t in grads.items():
            setattr(a, f, t.data_ptr())
        self.a, self.kind, self.d = a, kind, d
        self.dgrad_weights = dgrad_weights     # {"wt_qkv": W [out, in], ...}
        self.wt_of = None

    def _bind_wt(self):
        wt = TransposedWeights.active
        if wt is self.wt_of:
            return
        for f, W in self.dgrad_weights.items():
            img = wt.get(W, wait=False) if wt is not None else None
            setattr(self.a, f, 0 if img is None else img.data_ptr())
        self.wt_of = wt

    def sizes(self):
        a = self.a
        key = (a.kind, a.B, a.T, a.Tk, a.d, a.H, a.F)
        s = LayerCall._sizes.get(key)
        if s is None:
            offs = (ctypes.c_int64 * _lib.LAYER_NSLOT)()
            nb, mw, sw = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            call("mms2ut_layer_arena", ctypes.byref(a), offs, ctypes.byref(nb))
            call("mms2ut_layer_ws", ctypes.byref(a), ctypes.byref(mw), ctypes.byref(sw))
            s = (nb.value, list(offs), mw.value, sw.value, {})
            LayerCall._sizes[key] = s
        return s

    def fwd(self, x, B, T, self_len, seed, p, offs, Tk=0, cross_len=None, kv=None):
        """p = (p_drop, p_attn, p_act); offs = the six site offsets (mms2ut_layer order).
        Returns (arena uint8, byte offsets, argument snapshot)."""
        a = self.a
        a.B, a.T, a.Tk = B, T, Tk
        a.self_len = self_len.data_ptr()
        a.cross_len = cross_len.data_ptr() if cross_len is not None else 0
        a.kv, a.ld_kv = (kv.data_ptr(), kv.stride(0)) if kv is not None else (0, 0)
        a.p_drop, a.p_attn, a.p_act = p
        a.seed = seed
        a.off_sa_attn, a.off_sa_res, a.off_ca_attn, a.off_ca_res, a.off_act, a.off_ffn_res = offs
        a.x = x.data_ptr()
        self._bind_wt()
        nb, offsets, mw, _, _ = self.sizes()
        arena = torch.empty(nb, dtype=torch.uint8, device=x.device)
        a.saved = arena.data_ptr()
        ws = stream_workspace(mw, x.device)
        call("mms2ut_layer_fwd", ctypes.byref(a), None if ws is None else ws.data_ptr(), mw, _s())
        return arena, offsets, bytes(a)

    @staticmethod
    def view(arena, offsets, slot, shape, dtype=F16):
        n = 1
        for s in shape:
            n *= s
        o = offsets[slot]
        return arena[o:o + n * torch.tensor([], dtype=dtype).element_size()].view(dtype).view(shape)

    def bwd(self, snap, arena, dy, R, dy_drop=None, emit=None, dkv=None, last=False):
        """Backward of the forward whose argument snapshot is ``snap``.  emit = (p, (seed, offset)):
        also return dropout(dx) for the layer below.  last: nothing follows on the critical path
        (the weight gradients may take the whole chip).  Returns (dx, dropout(dx) or dx)."""
        emit_p, (emit_seed, emit_off) = (emit[0], emit[1]) if emit is not None and emit[0] > 0 else (0.0, (0, 0))
        nb, offsets, mw, sw, scr = self.sizes()
        sk = emit_p > 0
        s = scr.get(sk)
        if s is None:
            dxo, sb = (ctypes.c_int64 * 2)(), ctypes.c_int64()
            call("mms2ut_layer_scratch", ctypes.byref(self.a), float(emit_p), dxo, ctypes.byref(sb))
            s = scr[sk] = (sb.value, list(dxo))
        sbytes, dxo = s
        dev = dy.device
        scratch = torch.empty(sbytes, dtype=torch.uint8, device=dev)
        if TransposedWeights.active is not None:
            TransposedWeights.active.wait_ready()
        main_ws = stream_workspace(mw, dev)
        side = 0
        if _Side.enabled:
            side_stream(dev)
            side = _Side.ptr
            with _SIDE_REGION:
                side_ws = _workspace("layer_side", sw, dev)
        else:
            side_ws = _workspace("layer_side", sw, dev) if sw > 0 else None
        g = _lib.LAYER_GRAD_ARGS.pack(
            dy.data_ptr(), 0 if dy_drop is None else dy_drop.data_ptr(), float(emit_p), int(emit_seed),
            int(emit_off), 0 if dkv is None else dkv.data_ptr(), 0 if dkv is None else dkv.stride(0),
            scratch.data_ptr(), 0 if main_ws is None else main_ws.data_ptr(), mw,
            0 if side_ws is None else side_ws.data_ptr(), sw, 0 if last else SIDE_WGRAD_BLOCKS)
        call("mms2ut_layer_bwd", snap, g, _s(), side)
        if side:
            # the side stream reads the arena (saved activations), the scratch and the incoming
            # gradient (dy / its dropout: the grouped fc2 weight gradient runs after the layer's
            # whole dgrad chain): keep them until side_join; nothing else may reuse them before
            _Side.keep.extend((arena, scratch, dy) if dy_drop is None else (arena, scratch, dy, dy_drop))
            _Side.used = True
        d = self.d
        dx = scratch[dxo[0]:dxo[0] + 2 * R * d].view(F16).view(R, d)
        dxd = scratch[dxo[1]:dxo[1] + 2 * R * d].view(F16).view(R, d) if sk else dx
        return dx, dxd


class ConvCall:
    """The Conv1d subsampler enqueued by one library call each way (include/mms2ut.h
    mms2ut_conv1d_glu_fwd / _bwd: im2col, projection GEMM, GLU per layer from C++, the weight
    gradients on the side stream).  Weight / gradient / W^T pointers are bound once; each forward
    sets the batch shape and the arena and snapshots the argument block for its backward."""

    _sizes = {}

    def __init__(self, ks, couts, weights, biases, gweights, gbiases, dgrad_weights):
        a = _lib.ConvArgs()
        a.nlayers = len(ks)
        for i, k in enumerate(ks):
            a.k[i], a.cout[i] = k, couts[i]
            a.w[i], a.b[i] = weights[i].data_ptr(), biases[i].data_ptr()
            a.g_w[i], a.g_b[i] = gweights[i].data_ptr(), gbiases[i].data_ptr()
        self.a = a
        self.dgrad_weights = dgrad_weights     # {layer: W viewed [cout, C k]} for layers >= 1
        self.wt_of = None

    def _bind_wt(self):
        wt = TransposedWeights.active
        if wt is self.wt_of:
            return
        for i, W in self.dgrad_weights.items():
            img = wt.get(W, wait=False) if wt is not None else None
            self.a.wt[i] = 0 if img is None else img.data_ptr()
        self.wt_of = wt

    def sizes(self, a=None):
        """Arena / scratch / workspace sizes of the call described by `a` (the live argument block
        by default; a backward passes its forward's snapshot, which a later forward of the same
        call may have overwritten in self.a)."""
        a = self.a if a is None else a
        key = (a.B, a.T, a.C, a.nlayers, tuple(a.k), tuple(a.cout))
        s = ConvCall._sizes.get(key)
        if s is None:
            out_off, nb, sb, dxo = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            mw, sw = ctypes.c_int64(), ctypes.c_int64()
            call("mms2ut_conv1d_glu_arena", ctypes.byref(a), ctypes.byref(out_off), ctypes.byref(nb))
            call("mms2ut_conv1d_glu_scratch", ctypes.byref(a), ctypes.byref(dxo), ctypes.byref(sb))
            call("mms2ut_conv1d_glu_ws", ctypes.byref(a), ctypes.byref(mw), ctypes.byref(sw))
            s = (nb.value, out_off.value, sb.value, mw.value, sw.value)
            ConvCall._sizes[key] = s
        return s

    def fwd(self, x, B, T, C):
        """x [B*T, C] fp16 -> (arena, output [B*T_out, cout_last / 2] view, argument snapshot)."""
        a = self.a
        a.B, a.T, a.C = B, T, C
        a.x = x.data_ptr()
        self._bind_wt()
        nb, out_off, _, mw, _ = self.sizes()
        arena = torch.empty(nb, dtype=torch.uint8, device=x.device)
        a.saved = arena.data_ptr()
        ws = stream_workspace(mw, x.device)
        call("mms2ut_conv1d_glu_fwd", ctypes.byref(a), None if ws is None else ws.data_ptr(), mw, _s())
        Tout = T
        for i in range(a.nlayers):
            Tout = (Tout - 1) // 2 + 1
        Cg = a.cout[a.nlayers - 1] // 2
        out = arena[out_off:out_off + 2 * B * Tout * Cg].view(F16).view(B * Tout, Cg)
        return arena, out, bytes(a)

    def bwd(self, snap, arena, dy):
        """Backward of the forward whose argument snapshot is ``snap`` (weight / bias gradients)."""
        nb, _, sbytes, mw, sw = self.sizes(_lib.ConvArgs.from_buffer_copy(snap))
        dev = dy.device
        scratch = torch.empty(sbytes, dtype=torch.uint8, device=dev)
        if TransposedWeights.active is not None:
            TransposedWeights.active.wait_ready()
        main_ws = stream_workspace(mw, dev)
        side = 0
        if _Side.enabled:
            side_stream(dev)
            side = _Side.ptr
            with _SIDE_REGION:
                side_ws = _workspace("slab", sw, dev) if sw > 0 else None
        else:
            side_ws = _workspace("slab", sw, dev) if sw > 0 else None
        call("mms2ut_conv1d_glu_bwd", snap, dy.data_ptr(), scratch.data_ptr(),
             None if main_ws is None else main_ws.data_ptr(), mw, None if side_ws is None else side_ws.data_ptr(), sw,
             SIDE_WGRAD_BLOCKS if side else 0, _s(), side)
        if side:
            # the side stream reads the arena (im2col images) and the scratch (GLU gradients)
            _Side.keep.extend((arena, scratch, dy))
            _Side.used = True


class FusionCall:
    """The fusion tail (image LN, q / k|v projections, one-head attention, out-projection, sigmoid
    gate) enqueued by one library call each way (include/mms2ut.h mms2ut_gated_fusion_fwd / _bwd).
    Parameter / gradient / W^T pointers are bound once; each forward sets shapes, dropout sites and
    the arena and snapshots the argument block for its backward."""

    _sizes = {}

    def __init__(self, flags, params, grads, dgrad_weights):
        a = _lib.FusionArgs()
        for f, v in flags.items():
            setattr(a, f, v)
        for f, t in params.items():
            setattr(a, f, 0 if t is None else t.data_ptr())
        for f, t in grads.items():
            setattr(a, f, 0 if t is None else t.data_ptr())
        self.a = a
        self.dgrad_weights = dgrad_weights      # {"wt_q": W, ...}
        self.wt_of = None

    def _bind_wt(self):
        wt = TransposedWeights.active
        if wt is self.wt_of:
            return
        for f, W in self.dgrad_weights.items():
            img = wt.get(W, wait=False) if wt is not None else None
            setattr(self.a, f, 0 if img is None else img.data_ptr())
        self.wt_of = wt

    def sizes(self, want_dimg, a=None):
        """As ConvCall.sizes: `a` = a forward's argument snapshot (default: the live block)."""
        a = self.a if a is None else a
        key = (a.B, a.Te, a.Ti, a.Di, a.d, a.extra, a.gate, a.image_pre_norm, a.p_img > 0, a.p_txt > 0, a.p_attn > 0,
               bool(want_dimg))
        s = FusionCall._sizes.get(key)
        if s is None:
            oo, nb, sb, mw, sw = (ctypes.c_int64() for _ in range(5))
            so = (ctypes.c_int64 * 2)()
            call("mms2ut_gated_fusion_arena", ctypes.byref(a), ctypes.byref(oo), ctypes.byref(nb))
            call("mms2ut_gated_fusion_scratch", ctypes.byref(a), int(want_dimg), so, ctypes.byref(sb))
            call("mms2ut_gated_fusion_ws", ctypes.byref(a), ctypes.byref(mw), ctypes.byref(sw))
            s = (nb.value, oo.value, sb.value, list(so), mw.value, sw.value)
            FusionCall._sizes[key] = s
        return s

    def fwd(self, text, img, key_mask, B, Te, Ti, p, drops):
        """p = (p_img, p_txt, p_attn); drops = their (seed, offset) pairs or None.
        Returns (arena, output [B*Te, d] view, argument snapshot)."""
        a = self.a
        a.B, a.Te, a.Ti = B, Te, Ti
        a.p_img, a.p_txt, a.p_attn = p
        seeds = [dr[0] for dr in drops if dr is not None]
        a.seed = seeds[0] if seeds else 0
        assert all(sd == a.seed for sd in seeds), "one dropout seed per step"
        a.off_img, a.off_txt, a.off_attn = (dr[1] if dr is not None else 0 for dr in drops)
        a.key_mask, a.ld_mask = (key_mask.data_ptr(), key_mask.stride(0)) if key_mask is not None else (0, 0)
        a.text, a.img = text.data_ptr(), img.data_ptr()
        self._bind_wt()
        nb, oo, _, _, mw, _ = self.sizes(False)
        arena = torch.empty(nb, dtype=torch.uint8, device=text.device)
        a.saved = arena.data_ptr()
        ws = stream_workspace(mw, text.device)
        call("mms2ut_gated_fusion_fwd", ctypes.byref(a), None if ws is None else ws.data_ptr(), mw, _s())
        out = arena[oo:oo + 2 * B * Te * a.d].view(F16).view(B * Te, a.d)
        return arena, out, bytes(a)

    def bwd(self, snap, arena, keep, dres, want_dimg=False):
        """-> d(text) [B*Te, d] (and d(img) [B*Ti, Di] with want_dimg)."""
        a = _lib.FusionArgs.from_buffer_copy(snap)
        _, _, sbytes, so, mw, sw = self.sizes(want_dimg, a)
        dev = dres.device
        scratch = torch.empty(sbytes, dtype=torch.uint8, device=dev)
        if TransposedWeights.active is not None:
            TransposedWeights.active.wait_ready()
        main_ws = stream_workspace(mw, dev)
        side = 0
        if _Side.enabled:
            side_stream(dev)
            side = _Side.ptr
            with _SIDE_REGION:
                side_ws = _workspace("slab", sw, dev) if sw > 0 else None
        else:
            side_ws = _workspace("slab", sw, dev) if sw > 0 else None
        call("mms2ut_gated_fusion_bwd", snap, dres.data_ptr(), int(want_dimg), scratch.data_ptr(),
             None if main_ws is None else main_ws.data_ptr(), mw, None if side_ws is None else side_ws.data_ptr(), sw,
             SIDE_WGRAD_BLOCKS if side else 0, _s(), side)
        if side:
            _Side.keep.extend((arena, scratch, dres) + tuple(keep))
            _Side.used = True
        R, d = a.B * a.Te, a.d
        dtext = scratch[so[0]:so[0] + 2 * R * d].view(F16).view(R, d)
        if not want_dimg:
            return dtext
        Ri = a.B * a.Ti
        return dtext, scratch[so[1]:so[1] + 2 * Ri * a.Di].view(F16).view(Ri, a.Di)


def linear_dgrad(dy, W, out=None, *, epi=EPI_F16, aux=None, p=0.0, accumulate=False, drop=None):
    """dx[M,K] = dy[M,N] @ W[N,K]  (W row-major, reduction over N).  Reads the W^T image when one
    is registered (TransposedWeights), else W itself through transposed fragment reads.
    drop=(seed, offset): the forward dropout mask of the [M, K] output (EPI_GELU_DROP_BWD)."""
    M, N = dy.shape
    K = W.shape[1]
    if out is None:
        out = torch.empty(M, K, dtype=F16, device=dy.device)
    if accumulate:
        epi = EPI_F16_ACC
    seed, off = drop if (drop is not None and p > 0) else (0, 0)
    WT = TransposedWeights.active.get(W) if TransposedWeights.active is not None else None
    if WT is not None:
        gemm(dy, WT, out, M, K, N, a_kc=True, b_kc=True, lda=dy.stride(0), ldb=WT.stride(0),
             ldc=out.stride(0), epi=epi, aux=aux, ldaux=(aux.stride(0) if aux is not None else 0), p=p,
             seed=seed, offset=off, ld_rng=K)
        return out
    gemm(dy, W, out, M, K, N, a_kc=True, b_kc=False, lda=dy.stride(0), ldb=W.stride(0),
         ldc=out.stride(0), epi=epi, aux=aux, ldaux=(aux.stride(0) if aux is not None else 0), p=p,
         seed=seed, offset=off, ld_rng=K)
    return out


def _splitk_for(tiles, kred, slots=512):
    """split-K count for a weight gradient (reduction over kred token rows): the largest s whose
    tiles*s blocks still fit one round of the 512 block slots (2 per CU), so every block runs
    concurrently and no partial second round trails (round-2 scripts/wgrad_sweep.py, git history, isolated GEMM +
    slab reduction on the step's shapes: fc 3072x768 s3 vs the old fixed s8, qkv 2304x768 s4
    49 vs 60 us, cross-KV 9216x768 s1 174 vs 234 us; the 512-slot budget re-checked against
    256 / 1024 in round 2, profiles/round2_v3_wgrad_split_ab.txt).  Same rule as csrc/layers.hip."""
    s = max(1, min(16, slots // max(tiles, 1)))
    while s > 1 and kred // s < 256:
        s -= 1
    return s


class _Side:
    """Weight-gradient side stream: dW/db GEMMs and reductions do not feed the rest of the
    backward, so they run concurrently with the dgrad chain on a second HIP stream and fill the
    CUs the (latency-bound, dependent) dgrad kernels leave idle.

    The side region does not switch torch's current stream: kernels.py enqueues on
    ``override``.  Device memory read by side kernels (dy temporaries, saved activations) is kept
    referenced until ``side_join`` so the caching allocator cannot hand it to main-stream work
    before the side stream has consumed it; side-only scratch (split-K slabs, column partials)
    lives in persistent per-stream workspaces (the side stream serialises its own reuse)."""
    stream = None      # torch.cuda.Stream (RCCL buckets are enqueued on it, parallel.py)
    ptr = 0
    enabled = True     # False: side jobs run in order on the current stream (bench roofline pass)
    used = False
    override = 0
    keep = []
    ws = {}
    retain = False     # graph mode: regrown workspaces are retired, never freed (graphs bake pointers)
    retired = []


class _SideRegion:
    __slots__ = ()

    def __enter__(self):
        _Side.override = _Side.ptr
        return None

    def __exit__(self, *a):
        _Side.override = 0
        return False


_SIDE_REGION = _SideRegion()


class DevEvent:
    """A device-scope event (include/mms2ut.h mms2ut_event_*): orders work between this process's
    streams on one GPU without torch's system-scope fence (a full cache writeback per record,
    ~6 us of idle GPU each; profiles/round5_fork_fence.txt).  No timing, no host sync.  Owners
    re-record one event per use site; a wait binds to the record that precedes it."""
    __slots__ = ("h",)

    def __init__(self):
        h = ctypes.c_void_p()
        call("mms2ut_event_create", ctypes.addressof(h))
        self.h = h.value

    def record(self, stream):
        call("mms2ut_event_record", self.h, stream.cuda_stream)
        return self

    def wait(self, stream):
        call("mms2ut_event_wait", stream.cuda_stream, self.h)

    def __del__(self):
        try:
            if self.h:
                _lib.load().mms2ut_event_destroy(ctypes.c_void_p(self.h))
        except Exception:   # interpreter teardown
            pass


def stream_wait(waiter, signaler):
    """`waiter` waits for everything enqueued on `signaler` so far (device-scope event)."""
    if waiter.cuda_stream != signaler.cuda_stream:
        call("mms2ut_stream_wait", waiter.cuda_stream, signaler.cuda_stream)


_STREAMS = {}   # (device index, priority) -> ExternalStream, one per process


def make_stream(device, priority):
    """A non-blocking stream (include/mms2ut.h mms2ut_stream_create) wrapped for torch: work a
    caller leaves on the legacy NULL stream does not implicitly wait for it (measured equal to
    torch's pool streams in the bench, 17.05 vs 17.01-17.08 ms, round 4).  One stream per
    (device, priority) for the process: every Trainer reuses it, so building many trainers (test
    suites, tools) creates no more HIP streams (ExternalStream never destroys its handle; the cached
    ones are destroyed at exit, mms2ut_stream_destroy)."""
    dev = torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), int(priority))
    s = _STREAMS.get(key)
    if s is None:
        with torch.cuda.device(key[0]):
            h = ctypes.c_void_p()
            call("mms2ut_stream_create", int(priority), ctypes.addressof(h))
            s = torch.cuda.ExternalStream(h.value, device=dev)
        if not _STREAMS:
            atexit.register(_destroy_streams)
        _STREAMS[key] = s
    return s


def _destroy_streams():
    for s in _STREAMS.values():
        try:
            s.synchronize()
            _lib.load().mms2ut_stream_destroy(ctypes.c_void_p(s.cuda_stream))
        except Exception:   # interpreter teardown: the runtime may already be gone
            pass
    _STREAMS.clear()


def make_side_stream(device):
    """The weight-gradient side stream: lowest priority, so the hardware dispatcher prefers the
    critical path's workgroups (a CU-masked variant measured 5 % slower, round 1)."""
    return make_stream(device, 100)


def side_stream(device):
    """The (lazily created) weight-gradient side stream."""
    if _Side.stream is None:
        _Side.stream = make_side_stream(device)
        _Side.ptr = _Side.stream.cuda_stream
    return _Side.stream


def side_begin(*tensors):
    """Fork: the side stream waits for everything enqueued so far on the current stream."""
    if not _Side.enabled:
        return None
    if _Side.stream is None:
        _Side.stream = make_side_stream(_dev())
        _Side.ptr = _Side.stream.cuda_stream
    call("mms2ut_stream_wait", _Side.ptr, torch._C._cuda_getCurrentRawStream(_dev()))
    _Side.keep.extend(tensors)
    _Side.used = True
    return _SIDE_REGION


def wgrad_flush():
    """Launch a layer backward's deferred weight-gradient group now (mms2ut_wgrad_flush)."""
    call("mms2ut_wgrad_flush", torch._C._cuda_getCurrentRawStream(_dev()))


def side_join():
    """Join: the current stream waits for all side-stream work (before consuming gradients)."""
    if _Side.used and _Side.stream is not None:
        cur = torch._C._cuda_getCurrentRawStream(_dev())
        call("mms2ut_wgrad_flush", cur)   # a layer's deferred weight-gradient group, if any
        call("mms2ut_stream_wait", cur, _Side.ptr)
        _Side.used = False
        _Side.keep.clear()


def _workspace(key, numel, device, dtype=torch.float32):
    """Scratch owned by the stream it is used on (side-stream serialised reuse; regrowth keeps the
    old buffer alive until the next join)."""
    if _Side.override:
        buf = _Side.ws.get(key)
        if buf is None or buf.numel() < numel:
            if buf is not None:
                (_Side.retired if _Side.retain else _Side.keep).append(buf)
            buf = torch.empty(max(numel, 1 << 20), dtype=dtype, device=device)
            _Side.ws[key] = buf
        return buf[:numel]
    return torch.empty(numel, dtype=dtype, device=device)


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


_NULLCTX = _nullctx()


def _group_ok(dy, x, dW):
    N, K = dy.shape[1], x.shape[1]
    return (N % 8 == 0 and K % 8 == 0 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0 and
            dy.stride(1) == 1 and x.stride(1) == 1 and dW.is_contiguous() and
            all(t.data_ptr() % 16 == 0 for t in (dy, x, dW)) and
            dy.shape[0] * max(dy.stride(0), x.stride(0)) * 2 < 2 ** 31)


# grid cap of a grouped weight-gradient launch on the side stream (0: one block per tile).  A cap
# makes the launch persistent: 128 blocks held their slots for ~600 us per layer and pushed the
# critical path's 474-564-tile GEMMs into second rounds (22.4 ms per step against 18.1 uncapped
# or at 512, 18.5 with no side stream; profiles/round3_v1_side_blocks_ab.json).  Env
# MMS2UT_SIDE_WGRAD_BLOCKS overrides it (a multiple of 8; for A/B runs)
SIDE_WGRAD_BLOCKS = int(os.environ.get("MMS2UT_SIDE_WGRAD_BLOCKS", "0"))


def wgrad_group(problems, rows, max_blocks=0):
    """One grouped, unsplit weight-gradient launch (include/mms2ut.h mms2ut_wgrad_group):
    problems = [(dy [rows, N], x [rows, K], dW [N, K], db [N] or None), ...] (<= 8) on the current
    stream; dW / db overwritten; max_blocks > 0 caps the grid (persistent blocks)."""
    arr = (_lib.WgradArgs * len(problems))()
    for i, (dy, x, dW, db) in enumerate(problems):
        assert dy.shape[0] == rows and x.shape[0] == rows and tuple(dW.shape) == (dy.shape[1], x.shape[1])
        assert _group_ok(dy, x, dW), "wgrad_group: shapes / strides / alignment outside the kernel's rules"
        arr[i] = _lib.WgradArgs(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), dW.data_ptr(),
                                0 if db is None else db.data_ptr(), dy.shape[1], x.shape[1])
    call("mms2ut_wgrad_group", arr, len(problems), int(rows), int(max_blocks), _s())


def linear_wgrad(dy, x, dW, *, db=None, accumulate_f32=None, out_f32=None, side=True):
    """dW[N,K] (fp16 view into the flat grad buffer) = dy[M,N]^T @ x[M,K].
    With accumulate_f32 (an fp32 [N,K] buffer) the result is added there instead; with out_f32 it
    is written there in fp32.
    With db (fp16 [N]) the bias gradient sum_rows dy comes out of the same GEMM: its first column
    of tiles sums the dy rows it stages anyway.  A product with >= 256 output tiles (one per CU)
    runs unsplit through the grouped kernel (no fp32 slabs); smaller ones split K over the rows
    into fp32 slabs, reduced by one launch."""
    M, N = dy.shape
    K = x.shape[1]
    assert dW is None or tuple(dW.shape) == (N, K)
    if out_f32 is not None:
        assert accumulate_f32 is None and db is None and tuple(out_f32.shape) == (N, K)
        accumulate_f32 = out_f32     # the split-K slab path below, its reduction storing (mode 0)
    if accumulate_f32 is None and -(-N // 128) * -(-K // 128) >= 256 and _group_ok(dy, x, dW):
        ctx = side_begin(dy, x) if side else None
        with (ctx or _NULLCTX):
            wgrad_group([(dy, x, dW, db)], M, SIDE_WGRAD_BLOCKS if ctx is not None and _Side.enabled else 0)
        return dW
    if db is not None and (accumulate_f32 is not None or K % 64 or N % 4):
        linear_wgrad(dy, x, dW, accumulate_f32=accumulate_f32, side=side)
        return bias_grad(dy, db, side=side)
    ctx = side_begin(dy, x) if side else None
    with (ctx or _NULLCTX):
        tiles = -(-N // 128) * -(-K // 128)
        s = _splitk_for(tiles, M)
        slabs = _workspace("slab", s * N * K, dy.device)
        rs = _workspace("rowsum", s * N, dy.device) if db is not None else None
        gemm(dy, x, slabs, N, K, M, a_kc=False, b_kc=False, lda=dy.stride(0), ldb=x.stride(0), ldc=K,
             epi=EPI_F32, splitk=s, sCsplit=N * K, rowsum=rs, ld_rowsum=N)
        if db is not None and accumulate_f32 is None and N % 4 == 0:
            call("mms2ut_splitk_reduce_bias", slabs.data_ptr(), s, N * K, N, K, dW.data_ptr(), dW.stride(0),
                 rs.data_ptr(), db.data_ptr(), _s())
            return dW
        if db is not None:
            call("mms2ut_splitk_reduce", rs.data_ptr(), s, N, 1, N, db.data_ptr(), N, 1, 1.0, _s())
        if accumulate_f32 is not None:
            call("mms2ut_splitk_reduce", slabs.data_ptr(), s, N * K, N, K, accumulate_f32.data_ptr(),
                 accumulate_f32.stride(0), 0 if out_f32 is not None else 2, 1.0, _s())
            return accumulate_f32
        call("mms2ut_splitk_reduce", slabs.data_ptr(), s, N * K, N, K, dW.data_ptr(), dW.stride(0), 1,
             1.0, _s())
    return dW


def bias_grad(dy, db, accumulate=False, side=True):
    """db[N] = sum_rows dy[M,N] (fp16 out, fp32 accumulation)."""
    M, N = dy.shape
    L = _lib.load()
    ctx = side_begin(dy) if side else None
    with (ctx or _NULLCTX):
        nparts = L.mms2ut_colsum_nparts(M)
        part = _workspace("colsum", nparts * N, dy.device)
        call("mms2ut_colsum_f16", dy.data_ptr(), M, N, dy.stride(0), part.data_ptr(), nparts, _s())
        call("mms2ut_colsum_parts", part.data_ptr(), nparts, N, db.data_ptr(), int(accumulate), _s())
    return db

# ============================================================================ LayerNorm


def layernorm(x, g, b, eps=1e-5, *, out=None, grp=0, grp_out=0, p=0.0, drop=None):
    """y = LN(x).  With out/grp/grp_out/p the result goes to row (r // grp) * grp_out + r % grp of
    out (a padded layout) after dropout_p with the unpadded counters (layernorm_fwd_ex)."""
    R, D = x.shape
    mean = torch.empty(R, dtype=torch.float32, device=x.device)
    rstd = torch.empty(R, dtype=torch.float32, device=x.device)
    if out is None and not grp and p == 0.0:
        y = torch.empty_like(x)
        call("mms2ut_layernorm_fwd", x.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(),
             mean.data_ptr(), rstd.data_ptr(), R, D, eps, _s())
        return y, mean, rstd
    y = torch.empty_like(x) if out is None else out
    assert y.is_contiguous() and y.shape[-1] == D
    seed, off = drop if p > 0 else (0, 0)
    call("mms2ut_layernorm_fwd_ex", x.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(),
         mean.data_ptr(), rstd.data_ptr(), R, D, eps, int(grp), int(grp_out), float(p), seed, off, _s())
    return y, mean, rstd


def layernorm_bwd(dy, x, g, mean, rstd, dgb, dres=None, want_dx=True, emit=None, dy_grp=0, dy_grp_out=0,
                  dy_p=0.0, dy_drop=None, dgb_accumulate=False):
    """Returns dx (+dres). dgb: fp16 view of [dgamma | dbeta] (2*D contiguous), overwritten, or
    added to with dgb_accumulate (one LayerNorm applied at several places).
    emit=(p, (seed, offset)): also return dropout(dx) for the sublayer below -> (dx, dxd).
    dy_grp/dy_grp_out/dy_p: dy is read through layernorm(out=, grp=, p=)'s layout and dropout."""
    R, D = x.shape
    if dy_grp or dy_p > 0:
        assert emit is None and D % 256 == 0 and D <= 1024
        L = _lib.load()
        nparts = L.mms2ut_layernorm_bwd_nparts(R, D)
        part = torch.empty(nparts, 2 * D, dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x) if want_dx else None
        seed, off = dy_drop if dy_p > 0 else (0, 0)
        call("mms2ut_layernorm_bwd_ex", dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr(),
             rstd.data_ptr(), _p(dres), _p(dx), part.data_ptr(), R, D, None, 0.0, 0, 0, int(dy_grp),
             int(dy_grp_out), float(dy_p), seed, off, _s())
        ctx = side_begin(part)
        with (ctx or _NULLCTX):
            call("mms2ut_colsum_parts", part.data_ptr(), nparts, 2 * D, dgb.data_ptr(), 0, _s())
        return dx
    L = _lib.load()
    nparts = L.mms2ut_layernorm_bwd_nparts(R, D)
    part = torch.empty(nparts, 2 * D, dtype=torch.float32, device=x.device)
    dx = torch.empty_like(x) if want_dx else None
    dxd, p, seed, off = None, 0.0, 0, 0
    if emit is not None and emit[0] > 0:
        p, (seed, off) = emit
        dxd = torch.empty_like(x)
    call("mms2ut_layernorm_bwd", dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr(),
         rstd.data_ptr(), _p(dres), _p(dx), part.data_ptr(), R, D, _p(dxd), float(p), seed, off, _s())
    # gamma/beta gradients feed only the optimizer: their partial-sum reduction leaves the
    # critical path for the weight-gradient side stream
    ctx = side_begin(part)
    with (ctx or _NULLCTX):
        call("mms2ut_colsum_parts", part.data_ptr(), nparts, 2 * D, dgb.data_ptr(), int(dgb_accumulate), _s())
    if emit is not None:
        return dx, (dxd if dxd is not None else dx)
    return dx

# ============================================================================ attention


def attn_softmax(S, Z, H, Tq, Tk, ldS, key_len=None, key_mask=None, causal=False, extra_key=False,
                 p=0.0, drop=None):
    P = torch.empty_like(S)
    Pd = torch.empty_like(S) if p > 0 else P
    seed, off = drop if p > 0 else (0, 0)
    call("mms2ut_attn_softmax_fwd", S.data_ptr(), P.data_ptr(), Pd.data_ptr(), Z, H, Tq, Tk, ldS,
         _p(key_len), _p(key_mask), (key_mask.stride(0) if key_mask is not None else 0),
         int(causal), int(extra_key), float(p), seed, off, _s())
    return P, Pd


def attn_softmax_bwd(P, dPd, Z, H, Tq, Tk, ldS, p=0.0, drop=None, out=None):
    seed, off = drop if p > 0 else (0, 0)
    dS = dPd if out is None else out
    call("mms2ut_attn_softmax_bwd", P.data_ptr(), dPd.data_ptr(), dS.data_ptr(), Z, H, Tq, Tk, ldS,
         None, 0, 0, float(p), seed, off, _s())
    return dS

FLASH_HD = (64, 96, 128)


def _attn_args(q, k, v, o, ldq, ldk, ldv, ldo, B, H, Tq, Tk, hd, scale, key_len, causal, p, drop, lse,
               sq=0, sk=0, sv=0, so=0):
    """mms2ut_attn_args packed in one struct call (_lib.ATTN_ARGS, fields in AttnArgs order)."""
    seed, off = drop if p > 0 else (0, 0)
    return _lib.ATTN_ARGS.pack(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), ldq, ldk, ldv, ldo,
                               sq, sk, sv, so, B, H, Tq, Tk, hd, 0 if key_len is None else key_len.data_ptr(),
                               int(causal), scale, p, seed, off, lse.data_ptr())


def mha_fwd(q, k, v, o, ldq, ldk, ldv, ldo, B, H, Tq, Tk, hd, scale, key_len=None, causal=False,
            p=0.0, drop=None, sq=0, sk=0, sv=0, so=0):
    """Fused attention forward; returns the row log-sum-exp [B*H*Tq] (fp32) for the backward.
    s*: batch strides in elements (0 = rows of one batch follow each other: T * ld)."""
    lse = torch.empty(B * H * Tq, dtype=torch.float32, device=q.device)
    a = _attn_args(q, k, v, o, ldq, ldk, ldv, ldo, B, H, Tq, Tk, hd, scale, key_len, causal, p, drop, lse,
                   sq, sk, sv, so)
    call("mms2ut_mha_varlen_fwd", a, _s())
    return lse


def mha_bwd(q, k, v, o, ldq, ldk, ldv, ldo, B, H, Tq, Tk, hd, scale, key_len, causal, p, drop, lse,
            dout, lddo, dq, lddq, dk, lddk, dv, lddv):
    a = _attn_args(q, k, v, o, ldq, ldk, ldv, ldo, B, H, Tq, Tk, hd, scale, key_len, causal, p, drop, lse)
    Dd = torch.empty(B * H * Tq, dtype=torch.float32, device=q.device)
    call("mms2ut_mha_varlen_bwd", a, dout.data_ptr(), int(lddo), 0, Dd.data_ptr(), dq.data_ptr(),
         int(lddq), 0, dk.data_ptr(), int(lddk), 0, dv.data_ptr(), int(lddv), 0, _s())

# ============================================================================ elementwise


def dropout(x, p, drop, out=None):
    out = x if out is None else out
    if p <= 0:
        if out.data_ptr() != x.data_ptr():
            out.copy_(x)
        return out
    seed, off = drop
    call("mms2ut_dropout_fwd", x.data_ptr(), out.data_ptr(), x.numel(), float(p), seed, off, _s())
    return out


def dropout_mask(n, p, seed, offset, device):
    m = torch.empty(n, dtype=torch.uint8, device=device)
    call("mms2ut_dropout_mask", m.data_ptr(), n, float(p), int(seed), int(offset), _s())
    return m


def encoder_embed(h, pos_table, lens32, B, T, D, scale, p, drop):
    x = torch.empty_like(h)
    seed, off = drop if p > 0 else (0, 0)
    call("mms2ut_encoder_embed_fwd", h.data_ptr(), pos_table.data_ptr(), lens32.data_ptr(),
         x.data_ptr(), B, T, D, float(scale), float(p), seed, off, _s())
    return x


def scale_dropout_bwd(dx, scale, p, drop, out=None):
    out = torch.empty_like(dx) if out is None else out
    seed, off = drop if p > 0 else (0, 0)
    call("mms2ut_scale_dropout_bwd", dx.data_ptr(), out.data_ptr(), dx.numel(), float(scale),
         float(p), seed, off, _s())
    return out


def token_embed(tok, E, pos_table, B, T, D, pad, scale, p, drop):
    x = torch.empty(B * T, D, dtype=F16, device=E.device)
    seed, off = drop if p > 0 else (0, 0)
    call("mms2ut_token_embed_fwd", tok.data_ptr(), E.data_ptr(), pos_table.data_ptr(), x.data_ptr(),
         B, T, D, pad, float(scale), float(p), seed, off, _s())
    return x


def token_embed_bwd(tok, dx, dE32, B, T, D, pad, scale, p, drop):
    seed, off = drop if p > 0 else (0, 0)
    call("mms2ut_token_embed_bwd", tok.data_ptr(), dx.data_ptr(), dE32.data_ptr(), B, T, D, dE32.shape[0], pad,
         float(scale), float(p), seed, off, _s())


def add_f32_to_f16(a, b32, out):
    call("mms2ut_add_f32_to_f16", a.data_ptr(), b32.data_ptr(), out.data_ptr(), a.numel(), _s())
    return out


def add_f16(a, b, out=None):
    out = torch.empty_like(a) if out is None else out
    call("mms2ut_add_f16", a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), _s())
    return out


def glu(x, C):
    rows = x.shape[0]
    y = torch.empty(rows, C, dtype=F16, device=x.device)
    call("mms2ut_glu_fwd", x.data_ptr(), y.data_ptr(), rows, C, _s())
    return y


def glu_bwd(x, dy, C):
    rows = x.shape[0]
    dx = torch.empty(rows, 2 * C, dtype=F16, device=x.device)
    call("mms2ut_glu_bwd", x.data_ptr(), dy.data_ptr(), dx.data_ptr(), rows, C, _s())
    return dx


def im2col(x, B, Tin, Tout, C, k, stride=2, pad=None, ldcol=None):
    """col [B*Tout, ldcol] (ldcol >= C*k, zero columns past C*k)."""
    pad = k // 2 if pad is None else pad
    ldcol = C * k if ldcol is None else ldcol
    col = torch.empty(B * Tout, ldcol, dtype=F16, device=x.device)
    call("mms2ut_im2col_ld", x.data_ptr(), col.data_ptr(), B, Tin, Tout, C, k, stride, pad, ldcol, _s())
    return col


def col2im(dcol, B, Tin, Tout, C, k, stride=2, pad=None):
    pad = k // 2 if pad is None else pad
    dx = torch.empty(B * Tin, C, dtype=F16, device=dcol.device)
    call("mms2ut_col2im", dcol.data_ptr(), dx.data_ptr(), B, Tin, Tout, C, k, stride, pad, _s())
    return dx


def gate_bwd(dres, merge, g):
    R, D = dres.shape
    dpre = torch.empty_like(dres)
    dmerge = torch.empty(R, 2 * D, dtype=F16, device=dres.device)
    call("mms2ut_gate_bwd", dres.data_ptr(), merge.data_ptr(), g.data_ptr(), dpre.data_ptr(),
         dmerge.data_ptr(), R, D, _s())
    return dpre, dmerge


def copy2d(src, dst, rows, cols):
    call("mms2ut_copy2d", src.data_ptr(), src.stride(0), dst.data_ptr(), dst.stride(0), rows, cols,
         _s())

# ============================================================================ loss / optimizer


LS_XENT_PARTS = 512   # include/mms2ut.h MMS_LS_XENT_PARTS


def ls_xent_fwd(logits, ld, target, rows, V, eps, pad, loss_out, call_out=None):
    """loss_out[0:2] += {label-smoothed loss, nll} (fixed-order sum; loss_out may be None) and, with
    call_out, call_out[0:2] = this call's {loss, nll}; returns lse [rows]."""
    lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
    part = _workspace("ls_xent_part", 2 * LS_XENT_PARTS, logits.device)
    call("mms2ut_ls_xent_fwd_log", logits.data_ptr(), ld, target.data_ptr(), rows, V, float(eps), pad,
         lse.data_ptr(), part.data_ptr(), _p(loss_out), _p(call_out), _s())
    return lse


def set_f32(dst, vals):
    """dst[:len(vals)] = vals (fp32 device vector, <= 8 values) in one launch."""
    import ctypes
    arr = (ctypes.c_float * len(vals))(*[float(v) for v in vals])
    call("mms2ut_set_f32", dst.data_ptr(), len(vals), ctypes.addressof(arr), _s())


def ls_xent_bwd(logits, ld, target, rows, V, eps, pad, lse, grad, out):
    call("mms2ut_ls_xent_bwd", logits.data_ptr(), ld, target.data_ptr(), rows, V, float(eps), pad,
         lse.data_ptr(), grad.data_ptr(), out.data_ptr(), _s())
    return out


OST_MULT, OST_GNORM, OST_OVERFLOW, OST_STEP, OST_STEP_SIZE, OST_LOSS_SCALE, OST_ITER, \
    OST_LAST_OVERFLOW, OST_LAST_RESCALE, OST_CLIP_COEF, OST_FATAL, OST_LR, OST_INCONSISTENT = range(13)
OST_SIZE = 16


def grad_norm(grad, ost, sample_size=None, nparts=1024):
    part = torch.empty(nparts, dtype=torch.float32, device=grad.device)
    call("mms2ut_grad_sqnorm", grad.data_ptr(), grad.numel(), part.data_ptr(), nparts, _s())
    call("mms2ut_grad_norm_finalize", part.data_ptr(), nparts, ost.data_ptr(), _p(sample_size), _s())


def ctc_loss_fwd(logits, B, T, V, targets, in_len32, tgt_len32, max_tgt_len, blank, zero_infinity, loss_sum):
    """Adds the summed CTC loss to loss_sum (fp32 [1]); returns the workspace for ctc_loss_bwd."""
    import ctypes
    n = ctypes.c_int64()
    call("mms2ut_ctc_workspace_floats", int(B), int(T), int(max_tgt_len), ctypes.byref(n))
    work = torch.empty(max(n.value, 1), dtype=torch.float32, device=logits.device)
    assert targets.dtype == torch.int64 and in_len32.dtype == torch.int32 and tgt_len32.dtype == torch.int32
    call("mms2ut_ctc_loss_fwd", logits.data_ptr(), logits.stride(0), int(B), int(T), int(V), targets.data_ptr(),
         targets.stride(0), int(max_tgt_len), in_len32.data_ptr(), tgt_len32.data_ptr(), int(blank),
         int(zero_infinity), work.data_ptr(), loss_sum.data_ptr(), _s())
    return work


def ctc_loss_bwd(logits, B, T, V, targets, in_len32, tgt_len32, max_tgt_len, blank, work, grad_scale, out=None):
    out = torch.empty_like(logits) if out is None else out
    call("mms2ut_ctc_loss_bwd", logits.data_ptr(), logits.stride(0), int(B), int(T), int(V), targets.data_ptr(),
         targets.stride(0), int(max_tgt_len), in_len32.data_ptr(), tgt_len32.data_ptr(), int(blank), work.data_ptr(),
         grad_scale.data_ptr(), out.data_ptr(), out.stride(0), _s())
    return out


def grad_norm_check(buf, world, rank, ost, stage):
    call("mms2ut_grad_norm_check", buf.data_ptr(), int(world), int(rank), ost.data_ptr(), int(stage), _s())


def scale_f16(x, alpha):
    call("mms2ut_scale_f16", x.data_ptr(), x.numel(), float(alpha), _s())
    return x


_bound_seed = [None]


def bind_step_seed(delta):
    """Bind (or with None unbind) the device step-seed delta every dropout kernel adds to its seed
    (graph replay; include/mms2ut.h mms2ut_bind_step_seed).  Process-global; rebinding the bound
    tensor is free."""
    if delta is _bound_seed[0]:
        return
    if delta is not None:
        assert delta.is_cuda and delta.dtype == torch.int64 and delta.numel() == 1
    call("mms2ut_bind_step_seed", None if delta is None else delta.data_ptr())
    _bound_seed[0] = delta


def step_seed_advance(delta, inc):
    call("mms2ut_step_seed_advance", delta.data_ptr(), int(inc) & ((1 << 64) - 1), _s())


def accum_f16_f32(acc, x):
    assert acc.dtype == torch.float32 and x.dtype == F16 and acc.numel() == x.numel()
    call("mms2ut_accum_f16_f32", acc.data_ptr(), x.data_ptr(), x.numel(), _s())
    return acc


def optim_prepare(ost, lr, warmup_init_lr, warmup_updates, beta1, beta2, clip, scale_window, min_scale):
    call("mms2ut_optim_prepare", ost.data_ptr(), float(lr), float(warmup_init_lr), float(warmup_updates),
         float(beta1), float(beta2), float(clip), float(scale_window), float(min_scale), _s())


def adam(param, grad, master, m, v, ost, beta1, beta2, eps, wd):
    call("mms2ut_adam_fp16_master", param.data_ptr(), grad.data_ptr(), master.data_ptr(),
         m.data_ptr(), v.data_ptr(), param.numel(), ost.data_ptr(), float(beta1),
         float(beta2), float(eps), float(wd), _s())

# ============================================================================ fbank


def fbank(wave, wave_off, frame_off, total_frames, banks, mel_range, nbins=80):
    feats = torch.empty(total_frames, nbins, dtype=torch.float32, device=wave.device)
    B = wave_off.numel() - 1
    call("mms2ut_fbank_f32", wave.data_ptr(), wave_off.data_ptr(), frame_off.data_ptr(), B,
         total_frames, banks.data_ptr(), mel_range.data_ptr(), nbins, feats.data_ptr(), _s())
    return feats


CMVN_SPLIT = 8   # include/mms2ut.h MMS_CMVN_SPLIT


def cmvn_collate(feats, frame_off, B, Tmax, nbins=80, cmvn=True):
    out = torch.empty(B, Tmax, nbins, dtype=F16, device=feats.device)
    # include/mms2ut.h MMS_CMVN_WS_FLOATS: fp32 stats, then fp64 slice partials
    stats = torch.empty(((2 * B * nbins + 1) & ~1) + 2 * B * CMVN_SPLIT * 2 * nbins, dtype=torch.float32,
                        device=feats.device)
    call("mms2ut_fbank_cmvn_collate", feats.data_ptr(), frame_off.data_ptr(), B, Tmax, nbins,
         int(cmvn), stats.data_ptr(), out.data_ptr(), _s())
    return out


def specaugment(x, frame_off, masks, n_freq, n_time, mask_value=None):
    """In place on collated fp16 features x [B, Tmax, nbins]; masks int32 [B, 2*(n_freq+n_time)]
    on x's device (see include/mms2ut.h)."""
    B, Tmax, nbins = x.shape
    if masks.shape != (B, 2 * (n_freq + n_time)) or masks.dtype != torch.int32 or masks.device != x.device:
        raise ValueError(f"specaugment: masks {tuple(masks.shape)} {masks.dtype} for B={B}, {n_freq}+{n_time} masks")
    call("mms2ut_specaugment_f16", x.data_ptr(), frame_off.data_ptr(), B, Tmax, nbins, masks.data_ptr(),
         int(n_freq), int(n_time), int(mask_value is not None), float(mask_value or 0.0), _s())
    return x


def log_softmax_step(logits, V, pad, eos, mode=0, out=None):
    """fp32 [rows, V] = log_softmax(logits[:, :V].float()) with the beam-search step masks
    (mode 0: pad; 1: force eos; 2: forbid eos)."""
    rows = logits.shape[0]
    out = torch.empty(rows, V, dtype=torch.float32, device=logits.device) if out is None else out
    call("mms2ut_log_softmax_step", logits.data_ptr(), logits.stride(0), rows, int(V), int(pad), int(eos),
         int(mode), out.data_ptr(), _s())
    return out


def kv_cache_gather(src, dst, idx, rows):
    """dst[l, n, :rows] = src[l, idx[n], :rows] for caches [L, N, maxT, width] (idx int64 on device)."""
    L, Ns, T, W = src.shape
    Ld, N, Td, Wd = dst.shape
    if (L, T, W) != (Ld, Td, Wd) or idx.numel() != N or idx.dtype != torch.int64 or rows > T:
        raise ValueError(f"kv_cache_gather: src {tuple(src.shape)} dst {tuple(dst.shape)} idx {tuple(idx.shape)}")
    call("mms2ut_kv_cache_gather", src.data_ptr(), dst.data_ptr(), idx.data_ptr(), L, Ns, N, T, int(rows), W, _s())
    return dst


def decode_self_attn(q, cache_l, slot, N, H, hd, step_dev, kv_new, scale, out=None):
    """One decoder step of self-attention: cache_l [slots, maxT, 2*H*hd], slot int32 [>=N, maxT],
    step_dev int32 [1] (T = step + 1), kv_new [N, 2*H*hd] this step's K|V rows (stored into the cache)."""
    S, maxT, W = cache_l.shape
    if W != 2 * H * hd or slot.dtype != torch.int32 or slot.shape[1] != maxT or slot.shape[0] < N or S < N \
            or kv_new.shape[1] != W or step_dev.dtype != torch.int32:
        raise ValueError(f"decode_self_attn: cache {tuple(cache_l.shape)} slot {tuple(slot.shape)} N={N}")
    out = torch.empty(N, H * hd, dtype=F16, device=q.device) if out is None else out
    call("mms2ut_decode_self_attn", q.data_ptr(), q.stride(0), cache_l.data_ptr(), slot.data_ptr(), N, H, hd,
         maxT, step_dev.data_ptr(), kv_new.data_ptr(), kv_new.stride(0), W, out.data_ptr(), out.stride(0),
         float(scale), _s())
    return out


def decode_embed(tok, E, pos, step_dev, pad, N, D, scale, out=None):
    out = torch.empty(N, D, dtype=F16, device=E.device) if out is None else out
    call("mms2ut_decode_embed", tok.data_ptr(), E.data_ptr(), pos.data_ptr(), step_dev.data_ptr(), int(pad),
         out.data_ptr(), N, D, float(scale), _s())
    return out


def linear_splitk(x, W, bias=None, *, aux=None, relu=False, splitk=4, out=None):
    """out[M,N] = act(x @ W^T + bias) (+ aux) through `splitk` fp32 slabs and one reduction
    launch — for small-M GEMMs (the decoder step) whose dozen tiles would otherwise run long
    serial k-loops."""
    M, Kd = x.shape
    N = W.shape[0]
    out = torch.empty(M, N, dtype=F16, device=x.device) if out is None else out
    slabs = torch.empty(splitk, M, N, dtype=torch.float32, device=x.device)
    gemm(x, W, slabs, M, N, Kd, lda=x.stride(0), ldb=W.stride(0), ldc=N, epi=EPI_F32, splitk=splitk,
         sCsplit=M * N)
    call("mms2ut_splitk_epilogue_f16", slabs.data_ptr(), splitk, M * N, M, N, _p(bias), _p(aux),
         aux.stride(0) if aux is not None else 0, int(relu), out.data_ptr(), out.stride(0), _s())
    return out


def linear_splitk_ln(x, W, bias, aux, g, b, eps=1e-5, *, splitk=4):
    """(xo, y): xo = x @ W^T + bias + aux (split-K slabs), y = LayerNorm(xo) — one reduction launch."""
    M, Kd = x.shape
    N = W.shape[0]
    xo = torch.empty(M, N, dtype=F16, device=x.device)
    y = torch.empty(M, N, dtype=F16, device=x.device)
    slabs = torch.empty(splitk, M, N, dtype=torch.float32, device=x.device)
    gemm(x, W, slabs, M, N, Kd, lda=x.stride(0), ldb=W.stride(0), ldc=N, epi=EPI_F32, splitk=splitk,
         sCsplit=M * N)
    call("mms2ut_splitk_epilogue_ln_f16", slabs.data_ptr(), splitk, M * N, M, N, _p(bias), aux.data_ptr(),
         aux.stride(0), xo.data_ptr(), xo.stride(0), g.data_ptr(), b.data_ptr(), float(eps), y.data_ptr(),
         y.stride(0), _s())
    return xo, y


def beam_topk(lprobs, prev_col, bsz, beam, V, k, first_step):
    """(scores [bsz,k] f32, tokens [bsz,k] i64, beams [bsz,k] i64): top-k of lprobs + prev_col per
    sentence (prev_col: a strided fp32 column view [bsz*beam] of the cumulative scores)."""
    dev = lprobs.device
    sc = torch.empty(bsz, k, dtype=torch.float32, device=dev)
    tok = torch.empty(bsz, k, dtype=torch.int64, device=dev)
    bm = torch.empty(bsz, k, dtype=torch.int64, device=dev)
    ld = prev_col.stride(0) if prev_col is not None else 0
    work = torch.empty(bsz * 32 * k, dtype=torch.int64, device=dev)
    call("mms2ut_beam_topk", lprobs.data_ptr(), _p(prev_col), ld, bsz, beam, V, int(first_step), k,
         sc.data_ptr(), tok.data_ptr(), bm.data_ptr(), work.data_ptr(), _s())
    return sc, tok, bm


def round_up(x, m):
    return (x + m - 1) // m * m


__all__ = [n for n in dir() if not n.startswith("_")] + ["math"]
