"""Plain-Python restatement of fairseq's beam search — TEST INFRASTRUCTURE ONLY.

Follows fairseq ``SequenceGenerator._generate`` / ``BeamSearch.step`` / ``finalize_hypos`` /
``is_finished`` (the generator ``fairseq-generate --beam 10 --max-len-a 1`` builds for the
reference's S2UT model, mm_s2ut/scripts/textless/2_inference.sh:34-44; normalize_scores=True,
len_penalty, min_len=1, no unk penalty, no n-gram blocking, no prefix).  fairseq is absent from the
container (unpinned version): parity of the search is **unpinned** against fairseq
itself; this restatement is written per sentence with Python lists (independent of the product's
batched tensor bookkeeping) and the tests compare the two on identical step functions.

``step_fn(prefixes, live) -> lprobs``: prefixes is a list of token lists (each starting with eos),
beam per live sentence (``live``: the unfinished sentence ids in order); lprobs is a list of
per-vocabulary log-probabilities (python floats).  The
fp32 CPU decoder step ``full_recompute_step`` re-runs oracle/ref_model.decoder_forward over each
whole prefix (no incremental state), the independent check of the HIP incremental decoder.
"""
import math

import torch

from . import ref_model as R

NEG = -math.inf


def beam_search(step_fn, bsz, V, beam, max_len, pad=1, eos=2, min_len=1, len_penalty=1.0,
                normalize_scores=True):
    """Returns per sentence a list of {"tokens", "score", "positional_scores"} sorted by score."""
    cand_size = 2 * beam
    hyps = {s: [([eos], [])] * beam for s in range(bsz)}     # per live sentence: beam x (tokens, cum scores)
    ignore = {s: [False] * beam for s in range(bsz)}
    finalized = [[] for _ in range(bsz)]
    finished = [False] * bsz
    for step in range(max_len + 1):
        live = [s for s in range(bsz) if not finished[s]]
        prefixes = [h[0] for s in live for h in hyps[s]]
        lp_all = step_fn(prefixes, live)
        newly = []
        cands = {}
        for si, s in enumerate(live):
            rows = []
            for j in range(beam):
                lp = list(lp_all[si * beam + j])
                lp = [NEG if (x != x) else x for x in lp]
                lp[pad] = NEG
                if step >= max_len:
                    lp = [x if v == eos else NEG for v, x in enumerate(lp)]
                elif step < min_len:
                    lp[eos] = NEG
                rows.append(lp)
            flat = []
            for j in range(1 if step == 0 else beam):
                base = 0.0 if step == 0 else hyps[s][j][1][step - 1]
                for v in range(V):
                    flat.append((rows[j][v] + base, j * V + v))
            k = min(cand_size, len(flat) - 1)
            flat.sort(key=lambda t: (-t[0], t[1]))
            top = flat[:k]
            c = [(sc, idx // V, idx % V) for sc, idx in top]          # (score, beam, token)
            eos_mask = [tok == eos and sc != NEG for sc, _, tok in c]
            for pos in range(beam):
                if ignore[s][pos]:
                    eos_mask[pos] = False
            for pos in range(beam):
                if eos_mask[pos]:
                    sc, j, _ = c[pos]
                    toks = hyps[s][j][0][1:step + 1] + [eos]
                    cum = hyps[s][j][1][:step] + [sc]
                    ps = [cum[0]] + [cum[i] - cum[i - 1] for i in range(1, len(cum))]
                    score = sc / (step + 1) ** len_penalty if normalize_scores else sc
                    if len(finalized[s]) < beam:
                        finalized[s].append({"tokens": toks, "score": score, "positional_scores": ps})
            if any(eos_mask[:beam]) and not finished[s]:
                if len(finalized[s]) == beam or step == max_len:
                    newly.append(s)
            cands[s] = (c, eos_mask)
        for s in newly:
            finished[s] = True
        if all(finished) or step >= max_len:
            break
        for s in live:
            if finished[s]:
                continue
            c, eos_mask = cands[s]
            m = [ignore[s][p] or eos_mask[p] if p < beam else eos_mask[p] for p in range(len(c))]
            key = sorted(range(len(c)), key=lambda p: (m[p] * cand_size + p))
            act = key[:beam]
            ignore[s] = [(m[p] * cand_size + p) >= cand_size for p in act]
            new = []
            for p in act:
                sc, j, tok = c[p]
                toks, cum = hyps[s][j]
                new.append((toks[:step + 1] + [tok], cum[:step] + [sc]))
            hyps[s] = new
    for s in range(bsz):
        finalized[s].sort(key=lambda e: -e["score"])
    return finalized


def full_recompute_step(P, cfg, enc, enc_pad, beam, dtype=torch.float32):
    """step_fn over the fp32 oracle decoder: every prefix re-decoded from scratch.  enc [Te, B, d]
    time-major (oracle/ref_model.encoder_forward), enc_pad [B, Te]; hypothesis n belongs to
    sentence live[n // beam]."""

    def step(prefixes, live):
        n = len(prefixes)
        sent = [live[i // beam] for i in range(n)]
        T = len(prefixes[0])
        tok = torch.tensor(prefixes, dtype=torch.long)
        e = enc[:, sent]
        ep = enc_pad[sent]
        with torch.no_grad():
            logits = R.decoder_forward(P, tok, e, ep, cfg, dtype=dtype)
        lp = torch.log_softmax(logits[:, T - 1].float(), dim=-1)
        return lp.tolist()

    return step
