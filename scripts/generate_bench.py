"""Beam-search decoding throughput on the base model (random init, synthetic batch): the
fairseq-generate setting of scripts/textless/2_inference.sh:34-44 (--beam 10 --max-len-a 1,
max_len_b 200).  Random weights rarely emit </s>, so every sentence runs to max_len: a worst-case
(longest) decode.  Prints one JSON line: decoder steps/s, hypothesis-tokens/s, ms per step.

usage: python scripts/generate_bench.py [--bsz 16] [--frames 300] [--beam 10] [--max-len-b 200]
"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mm = importlib.import_module("multimodal-s2ut_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bsz", type=int, default=16)
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--beam", type=int, default=10)
    ap.add_argument("--max-len-a", type=float, default=1.0)
    ap.add_argument("--max-len-b", type=int, default=200)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    cfg = mm.default_cfg()
    model = mm.MMS2UTModel(cfg, device="cuda:0").init_params(seed=1)
    sample = mm.data.make_sample([a.frames] * a.bsz, [10] * a.bsz, img_tokens=577, img_dim=768, seed=0)
    batch = mm.runtime.prepare_batch(sample, model.cfg, "cuda:0")
    out = None
    for r in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hyps = mm.generate.generate(model, batch, beam_size=a.beam, max_len_a=a.max_len_a, max_len_b=a.max_len_b)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = max(len(h["tokens"]) for hs in hyps for h in hs)
        if r > 0:
            out = dt if out is None else min(out, dt)
    hyp_tokens = steps * a.bsz * a.beam
    print(json.dumps({"metric": "beam-search decode", "bsz": a.bsz, "beam": a.beam, "src_frames": a.frames,
                      "steps": steps, "s_per_batch": out, "ms_per_step": 1e3 * out / steps,
                      "hyp_tokens_per_s": hyp_tokens / out, "sentences_per_s": a.bsz / out,
                      "note": "random weights: every sentence decodes to max_len (worst case)"}))


if __name__ == "__main__":
    main()
