"""Beam-search inference over the unit decoder: ``fairseq-generate --beam 10
--max-len-a 1`` (mm_s2ut/scripts/textless/2_inference.sh:34-44) on the HIP path.

Two parts:

* ``IncrementalDecoder`` — fairseq ``TransformerDecoder`` with ``incremental_state``: one new
  token per hypothesis per step.  Every layer's self-attention K|V rows live in a cache
  [L_d, slots, maxT, 2d]: the layer's one Q|K|V projection yields this step's K|V rows, and
  ``decode_self_attn`` stores them as row `step` of slot n while it attends.  Rows never move:
  a slot table [N, maxT] int32 says which slot holds row t of hypothesis n, so
  ``reorder_incremental_state`` permutes N·step indices instead of copying every layer's K/V
  (fairseq's index_select of the cache), and the attention reads K/V through the table (one
  256-thread block per hypothesis·head).  The step reads its position from a device counter, so
  it replays as one HIP graph.  Cross-attention K/V of all layers are one GEMM over the encoder
  output at the start
  (the training path's batched slab); they stay per *sentence*: the beam hypotheses of sentence s
  are the query rows [s·beam, (s+1)·beam) of one attention problem (B = sentences, Tq = beam), so
  nothing is expanded by the beam (``reorder_encoder_out`` is the identity within a sentence and
  a sentence-row gather when finished sentences leave the batch).  Final LN, tied-embedding
  logits GEMM, then ``log_softmax_step`` (log_softmax of the fp16 logits in fp32 fused with the
  step's pad / eos masking).
* ``SequenceGenerator`` — fairseq ``SequenceGenerator._generate`` + ``BeamSearch.step`` +
  ``finalize_hypos`` (normalize_scores, len_penalty, min_len 1, no unk penalty / n-gram blocking /
  prefix / constraints), as device tensor bookkeeping in torch around the decoder above.  Works with
  any decoder object exposing ``step(tokens_last, step, mode)`` / ``reorder(state, batch_idxs)``
  (the CPU tests drive it with a toy decoder against oracle/ref_generate.py).
"""
import math
import os

import torch

from . import kernels as K
from .kernels import F16

MODE_NONE, MODE_FORCE_EOS, MODE_NO_EOS = 0, 1, 2


def _lin(x, W, b, *, aux=None, relu=False, out=None):
    """Decoder-step projection: split-K over fp32 slabs when the hypothesis rows leave most of the
    chip idle (tiles * s <= ~256 blocks, k-chunks >= 256), else the fused-epilogue GEMM."""
    M, Kd = x.shape
    N = W.shape[0]
    tiles = -(-M // 128) * -(-N // 128)
    s = min(8, max(1, 256 // tiles), Kd // 256)
    if s > 1:
        return K.linear_splitk(x, W, b, aux=aux, relu=relu, splitk=s, out=out)
    if aux is not None:
        return K.linear(x, W, b, out=out, epi=K.EPI_DROP_RESID, aux=aux, p=0.0)
    return K.linear(x, W, b, out=out, epi=K.EPI_RELU_DROP if relu else K.EPI_F16, p=0.0)


def _lin_ln(x, W, b, aux, g, beta):
    """(x_out, LN(x_out)) for a residual projection followed by a LayerNorm: one split-K reduction
    launch that also normalises when split-K applies (bit-identical to _lin + layernorm)."""
    M, Kd = x.shape
    N = W.shape[0]
    tiles = -(-M // 128) * -(-N // 128)
    s = min(8, max(1, 256 // tiles), Kd // 256)
    if s > 1 and N <= 1024:
        return K.linear_splitk_ln(x, W, b, aux, g, beta, splitk=s)
    xo = _lin(x, W, b, aux=aux)
    return xo, K.layernorm(xo, g, beta)[0]


class IncrementalDecoder:
    def __init__(self, model, enc, enc_len32, Te, bsz, beam, max_len, graphs=None):
        """enc [bsz*Te, d] fp16 (rows b*Te + t, the encoder's output incl. fusion), enc_len32 [bsz]."""
        self.m = model
        cfg = model.cfg
        self.d, self.H, self.L = cfg["decoder_embed_dim"], cfg["decoder_attention_heads"], cfg["decoder_layers"]
        self.V, self.pad, self.eos = cfg["vocab_size"], cfg["padding_idx"], 2
        self.hd = self.d // self.H
        if self.hd not in K.FLASH_HD:
            raise NotImplementedError(f"incremental decoding needs head dim in {K.FLASH_HD}, got {self.hd}")
        self.beam, self.Te = beam, Te
        self.bsz = bsz
        self.maxT = max_len + 2
        dev = enc.device
        self.dev = dev
        model.params.await_all()
        Wkv, bkv = model.cross_kv()
        self.kv_all = K.linear(enc, Wkv, bkv)            # [bsz*Te, L*2d]
        self.enc_len32 = enc_len32
        N = bsz * beam
        self.cache = torch.empty(self.L, N, self.maxT, 2 * self.d, dtype=F16, device=dev)
        self.slot = torch.zeros(N, self.maxT, dtype=torch.int32, device=dev)
        self.slot_tmp = torch.empty_like(self.slot)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tok = torch.zeros(N, dtype=torch.long, device=dev)
        self.pos = model._ensure_pos(self.maxT + 2, "dec")
        self.scale = 1.0 if cfg["no_scale_embedding"] else math.sqrt(self.d)
        self.Vp = K.round_up(self.V, 64)
        self.logits = torch.empty(N, self.Vp, dtype=F16, device=dev)
        self.step_no = 0
        # the decoder step is ~100 launches of fixed shapes: replay it as one HIP graph (recaptured
        # when finished sentences shrink the batch); MMS2UT_DECODE_GRAPH=0 runs it eagerly
        if graphs is None:
            graphs = os.environ.get("MMS2UT_DECODE_GRAPH", "1") != "0"
        self.use_graphs = graphs
        self.graph = None
        self.eager_steps = 0

    @property
    def N(self):
        return self.bsz * self.beam

    def reorder(self, reorder_state, batch_idxs=None):
        """reorder_incremental_state(reorder_state) + reorder_encoder_out: reorder_state [N_new]
        indexes the current hypotheses (fairseq's corrected index into the previous batch).
        Cache rows are write-once (row `step` of slot n is fresh at every step), so surviving
        hypotheses keep referencing their ancestors' rows wherever they live: only the slot table
        moves (in place while the batch keeps its size, so a captured step graph stays valid)."""
        if batch_idxs is None:
            torch.index_select(self.slot, 0, reorder_state, out=self.slot_tmp)
            self.slot.copy_(self.slot_tmp)
            return
        self.slot = self.slot.index_select(0, reorder_state)
        self.slot_tmp = torch.empty_like(self.slot)
        nb = batch_idxs.numel()
        kv = torch.empty(nb * self.Te, self.kv_all.shape[1], dtype=F16, device=self.dev)
        K.kv_cache_gather(self.kv_all.view(1, self.bsz, self.Te, -1), kv.view(1, nb, self.Te, -1),
                          batch_idxs.to(torch.int64), self.Te)
        self.kv_all = kv
        self.enc_len32 = self.enc_len32.index_select(0, batch_idxs)
        self.bsz = nb
        self.tok = torch.zeros(self.N, dtype=torch.long, device=self.dev)
        self.logits = torch.empty(self.N, self.Vp, dtype=F16, device=self.dev)
        self.graph = None
        self.eager_steps = 0

    def _body(self):
        """One decoder step over the static buffers (tok, step_dev, slot, cache) -> self.logits."""
        m, d, H, hd, N = self.m, self.d, self.H, self.hd, self.N
        x = K.decode_embed(self.tok, m.P("decoder.embed_tokens.weight"), self.pos, self.step_dev, self.pad, N, d,
                           self.scale)
        h1, _, _ = K.layernorm(x, m.P("decoder.layers.0.self_attn_layer_norm.weight"),
                               m.P("decoder.layers.0.self_attn_layer_norm.bias"))
        for l in range(self.L):
            p = f"decoder.layers.{l}"
            # one Q|K|V projection (the weights are adjacent in the flat buffer); K|V are this step's
            # cache rows, which the attention kernel stores
            Wqkv = m.params.span(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight").view(3 * d, d)
            bqkv = m.params.span(p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias")
            qkv = _lin(h1, Wqkv, bqkv)
            O = K.decode_self_attn(qkv[:, :d], self.cache[l], self.slot, N, H, hd, self.step_dev, qkv[:, d:],
                                   hd ** -0.5)
            x2, h2 = _lin_ln(O, m.P(p + ".self_attn.out_proj.weight"), m.P(p + ".self_attn.out_proj.bias"), x,
                             m.P(p + ".encoder_attn_layer_norm.weight"), m.P(p + ".encoder_attn_layer_norm.bias"))
            q2 = _lin(h2, m.P(p + ".encoder_attn.q_proj.weight"), m.P(p + ".encoder_attn.q_proj.bias"))
            kv = self.kv_all[:, 2 * d * l:2 * d * (l + 1)]
            ldkv = self.kv_all.stride(0)
            O2 = torch.empty(N, d, dtype=F16, device=self.dev)
            K.mha_fwd(q2, kv, kv[:, d:], O2, d, ldkv, ldkv, d, self.bsz, H, self.beam, self.Te, hd, hd ** -0.5,
                      key_len=self.enc_len32)
            x3, h3 = _lin_ln(O2, m.P(p + ".encoder_attn.out_proj.weight"), m.P(p + ".encoder_attn.out_proj.bias"),
                             x2, m.P(p + ".final_layer_norm.weight"), m.P(p + ".final_layer_norm.bias"))
            f1 = _lin(h3, m.P(p + ".fc1.weight"), m.P(p + ".fc1.bias"), relu=True)
            nxt = f"decoder.layers.{l + 1}.self_attn_layer_norm" if l + 1 < self.L else "decoder.layer_norm"
            x, h1 = _lin_ln(f1, m.P(p + ".fc2.weight"), m.P(p + ".fc2.bias"), x3, m.P(nxt + ".weight"),
                            m.P(nxt + ".bias"))
        xl = h1                                      # the decoder's final LayerNorm
        K.gemm(xl, m.P("decoder.embed_tokens.weight"), self.logits, N, self.V, d, lda=d, ldb=d, ldc=self.Vp)

    def beam_topk(self, lprobs, prev_col, bsz, beam, V, k, first_step):
        return K.beam_topk(lprobs, prev_col, bsz, beam, V, k, first_step)

    def step(self, tokens_last, step, mode=MODE_NONE):
        """tokens_last [N] int64 (the token at position `step` of every hypothesis) -> lprobs [N, V]."""
        assert self.step_no == step and self.slot.shape[0] == self.N and step + 1 < self.maxT
        self.tok.copy_(tokens_last)
        self.step_dev.fill_(step)
        if self.graph is not None:
            self.graph.replay()
        elif self.use_graphs and self.eager_steps >= 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._body()
            self.graph = g
            g.replay()
        else:
            self._body()
            self.eager_steps += 1
        self.step_no += 1
        return K.log_softmax_step(self.logits, self.V, self.pad, self.eos, mode)


class SequenceGenerator:
    """fairseq SequenceGenerator (beam search) over a step/reorder decoder."""

    def __init__(self, beam_size=10, max_len_a=1.0, max_len_b=200, max_len=3000, min_len=1,
                 normalize_scores=True, len_penalty=1.0, pad=1, eos=2):
        self.beam = beam_size
        self.max_len_a, self.max_len_b, self.max_len = max_len_a, max_len_b, max_len
        self.min_len, self.normalize_scores, self.len_penalty = min_len, normalize_scores, len_penalty
        self.pad, self.eos = pad, eos

    def max_steps(self, src_len):
        """max_len = min(a·src_len + b, max_len - 1) (src_len: padded source frames)."""
        return min(int(self.max_len_a * src_len + self.max_len_b), self.max_len - 1)

    def generate(self, decoder, bsz, max_len, V, device):
        beam, pad, eos = self.beam, self.pad, self.eos
        N = bsz * beam
        scores = torch.zeros(N, max_len + 1, dtype=torch.float32, device=device)
        tokens = torch.full((N, max_len + 2), pad, dtype=torch.long, device=device)
        tokens[:, 0] = eos
        cands_to_ignore = torch.zeros(bsz, beam, dtype=torch.bool, device=device)
        finalized = [[] for _ in range(bsz)]
        finished = [False] * bsz
        num_remaining = bsz
        cand_size = 2 * beam
        bbsz_offsets = (torch.arange(bsz, device=device) * beam).unsqueeze(1)
        cand_offsets = torch.arange(cand_size, device=device)
        reorder_state, batch_idxs = None, None
        for step in range(max_len + 1):
            if reorder_state is not None:
                if batch_idxs is not None:
                    corr = batch_idxs - torch.arange(batch_idxs.numel(), device=device)
                    reorder_state.view(-1, beam).add_(corr.unsqueeze(-1) * beam)
                decoder.reorder(reorder_state, batch_idxs)
            mode = MODE_FORCE_EOS if step >= max_len else (MODE_NO_EOS if step < self.min_len else MODE_NONE)
            lprobs = decoder.step(tokens[:, step], step, mode)
            # BeamSearch.step
            k = min(cand_size, (1 if step == 0 else beam) * V - 1)
            if hasattr(decoder, "beam_topk"):     # HIP selection kernel (ties to the lower flat index)
                cand_scores, cand_indices, cand_beams = decoder.beam_topk(
                    lprobs, None if step == 0 else scores[:, step - 1], bsz, beam, V, k, step == 0)
            else:
                lp = lprobs.view(bsz, beam, V)
                if step == 0:
                    lp = lp[:, ::beam, :].contiguous()
                else:
                    lp = lp + scores.view(bsz, beam, -1)[:, :, step - 1].unsqueeze(-1)
                cand_scores, idx = torch.topk(lp.view(bsz, -1), k=k)
                cand_beams = torch.div(idx, V, rounding_mode="trunc")
                cand_indices = idx.fmod(V)
            cand_bbsz_idx = cand_beams.add(bbsz_offsets)
            eos_mask = cand_indices.eq(eos) & cand_scores.ne(-math.inf)
            eos_mask[:, :beam][cands_to_ignore] = False
            eos_bbsz_idx = torch.masked_select(cand_bbsz_idx[:, :beam], mask=eos_mask[:, :beam])
            finalized_sents = []
            if eos_bbsz_idx.numel() > 0:
                eos_scores = torch.masked_select(cand_scores[:, :beam], mask=eos_mask[:, :beam])
                finalized_sents = self._finalize(step, eos_bbsz_idx, eos_scores, tokens, scores, finalized,
                                                 finished, max_len)
                num_remaining -= len(finalized_sents)
            if num_remaining == 0 or step >= max_len:
                break
            if finalized_sents:
                new_bsz = bsz - len(finalized_sents)
                batch_mask = torch.ones(bsz, dtype=torch.bool, device=device)
                batch_mask[torch.tensor(finalized_sents, device=device)] = False
                batch_idxs = torch.arange(bsz, device=device).masked_select(batch_mask)
                eos_mask = eos_mask[batch_idxs]
                cand_beams = cand_beams[batch_idxs]
                bbsz_offsets = bbsz_offsets[:new_bsz]
                cand_bbsz_idx = cand_beams.add(bbsz_offsets)
                cand_scores = cand_scores[batch_idxs]
                cand_indices = cand_indices[batch_idxs]
                cands_to_ignore = cands_to_ignore[batch_idxs]
                scores = scores.view(bsz, -1)[batch_idxs].view(new_bsz * beam, -1)
                tokens = tokens.view(bsz, -1)[batch_idxs].view(new_bsz * beam, -1)
                bsz = new_bsz
            else:
                batch_idxs = None
            eos_mask[:, :beam] = ~((~cands_to_ignore) & (~eos_mask[:, :beam]))
            active_mask = torch.add(eos_mask.type_as(cand_offsets) * cand_size, cand_offsets[: eos_mask.size(1)])
            new_ignore, active_hypos = torch.topk(active_mask, k=beam, dim=1, largest=False)
            cands_to_ignore = new_ignore.ge(cand_size)[:, :beam]
            active_bbsz_idx = torch.gather(cand_bbsz_idx, 1, active_hypos).view(-1)
            active_scores = torch.gather(cand_scores, 1, active_hypos)
            tokens[:, : step + 1] = torch.index_select(tokens[:, : step + 1], 0, active_bbsz_idx)
            tokens.view(bsz, beam, -1)[:, :, step + 1] = torch.gather(cand_indices, 1, active_hypos)
            if step > 0:
                scores[:, :step] = torch.index_select(scores[:, :step], 0, active_bbsz_idx)
            scores.view(bsz, beam, -1)[:, :, step] = active_scores
            reorder_state = active_bbsz_idx
        for s in range(len(finalized)):
            sc = torch.tensor([float(e["score"]) for e in finalized[s]])
            order = torch.sort(sc, descending=True)[1].tolist()
            finalized[s] = [finalized[s][i] for i in order]
        return finalized

    def _finalize(self, step, bbsz_idx, eos_scores, tokens, scores, finalized, finished, max_len):
        beam = self.beam
        tokens_clone = tokens.index_select(0, bbsz_idx)[:, 1: step + 2]
        tokens_clone[:, step] = self.eos
        pos_scores = scores.index_select(0, bbsz_idx)[:, : step + 1]
        pos_scores[:, step] = eos_scores
        pos_scores[:, 1:] = pos_scores[:, 1:] - pos_scores[:, :-1]
        if self.normalize_scores:
            eos_scores = eos_scores / (step + 1) ** self.len_penalty
        cum_unfin, prev = [], 0
        for f in finished:
            if f:
                prev += 1
            else:
                cum_unfin.append(prev)
        unfin_idx = torch.div(bbsz_idx, beam, rounding_mode="trunc").tolist()
        sent = [u + cum_unfin[u] for u in unfin_idx]
        toks, sc, ps = tokens_clone.cpu(), eos_scores.cpu(), pos_scores.cpu()
        for i in range(len(sent)):
            if len(finalized[sent[i]]) < beam:
                finalized[sent[i]].append({"tokens": toks[i], "score": float(sc[i]), "positional_scores": ps[i]})
        newly = []
        for s, u in sorted(set(zip(sent, unfin_idx))):
            if not finished[s] and (len(finalized[s]) == beam or step == max_len):
                finished[s] = True
                newly.append(u)
        return newly


def generate(model, batch, beam_size=10, max_len_a=1.0, max_len_b=200, max_len=None, len_penalty=1.0,
             min_len=1):
    """fairseq-generate on one DeviceBatch: encoder (eval, fusion included) -> beam search.
    Returns, per sentence in batch order, the hypotheses sorted by score (fairseq's dicts)."""
    was = model.training
    model.eval()
    try:
        enc, enc_len32, Te, _ = model.encoder_forward(batch)
        bsz = batch.src.shape[0]
        gen = SequenceGenerator(beam_size, max_len_a, max_len_b,
                                max_len or model.cfg["max_target_positions"], min_len=min_len,
                                len_penalty=len_penalty, pad=model.cfg["padding_idx"])
        T = gen.max_steps(batch.src.shape[1])
        dec = IncrementalDecoder(model, enc, enc_len32, Te, bsz, beam_size, T)
        return gen.generate(dec, bsz, T, model.cfg["vocab_size"], enc.device)
    finally:
        model.train(was)
