"""CPU: the product's batched beam search (generate.SequenceGenerator, fairseq SequenceGenerator
semantics) against the per-sentence Python restatement (oracle/ref_generate.beam_search) on the
same deterministic toy decoder: identical hypotheses (tokens bit-exact, scores to fp32 rounding),
including finished sentences leaving the batch, max-length forcing and min_len."""
import math
import random

import pytest
import torch

from conftest import pkg
from oracle import ref_generate as RG

PAD, EOS = 1, 2


def toy_logits(sent, prefix, V, sharp):
    r = random.Random(hash((sent, len(prefix)) + tuple(prefix)))
    z = [sharp * r.gauss(0.0, 1.0) for _ in range(V)]
    z[EOS] += 0.6 * len(prefix) - 3.0          # hypotheses end at varied lengths
    m = max(z)
    lse = m + math.log(sum(math.exp(v - m) for v in z))
    return [v - lse for v in z]


class ToyDecoder:
    """The product decoder interface (step / reorder) over toy_logits, masks as log_softmax_step."""

    def __init__(self, bsz, beam, V, sharp):
        self.pref = [[] for _ in range(bsz * beam)]
        self.sent = list(range(bsz))
        self.beam, self.V, self.sharp = beam, V, sharp

    def reorder(self, state, batch_idxs=None):
        self.pref = [list(self.pref[i]) for i in state.tolist()]
        if batch_idxs is not None:
            self.sent = [self.sent[i] for i in batch_idxs.tolist()]

    def step(self, tokens_last, step, mode):
        rows = []
        for n, t in enumerate(tokens_last.tolist()):
            self.pref[n].append(t)
            lp = toy_logits(self.sent[n // self.beam], self.pref[n], self.V, self.sharp)
            lp[PAD] = -math.inf
            if mode == 1:
                lp = [x if v == EOS else -math.inf for v, x in enumerate(lp)]
            elif mode == 2:
                lp[EOS] = -math.inf
            rows.append(lp)
        return torch.tensor(rows, dtype=torch.float32)


@pytest.mark.parametrize("bsz,beam,V,max_len,sharp,lenpen", [
    (3, 4, 23, 9, 1.5, 1.0), (2, 10, 40, 14, 2.0, 1.0), (4, 2, 11, 6, 1.0, 0.5), (1, 3, 17, 1, 1.0, 1.0)])
def test_beam_search_matches_restatement(bsz, beam, V, max_len, sharp, lenpen):
    G = pkg("generate")
    gen = G.SequenceGenerator(beam_size=beam, len_penalty=lenpen)
    got = gen.generate(ToyDecoder(bsz, beam, V, sharp), bsz, max_len, V, torch.device("cpu"))

    def step_fn(prefixes, live):
        return [toy_logits(live[i // beam], p, V, sharp) for i, p in enumerate(prefixes)]

    ref = RG.beam_search(step_fn, bsz, V, beam, max_len, len_penalty=lenpen)
    assert len(got) == len(ref) == bsz
    for s in range(bsz):
        assert len(got[s]) == len(ref[s]) == beam
        for g, r in zip(got[s], ref[s]):
            assert g["tokens"].tolist() == r["tokens"]
            assert g["tokens"][-1] == EOS and len(g["tokens"]) <= max_len + 1
            assert math.isclose(g["score"], r["score"], rel_tol=1e-5, abs_tol=1e-5)
            assert torch.allclose(g["positional_scores"], torch.tensor(r["positional_scores"]), atol=1e-4)


def test_max_steps_rule():
    G = pkg("generate")
    gen = G.SequenceGenerator(beam_size=10, max_len_a=1.0, max_len_b=200, max_len=3000)
    assert gen.max_steps(500) == 700                  # a*src_len + b
    assert gen.max_steps(5000) == 2999                # capped by max_decoder_positions - 1
