"""Localise the HIP-vs-oracle gradient error: the smoke configuration (tiny
2+2, conv 256, no dropout) and the base configuration, backward at loss scale 1 (what the smoke
test used) and at the fp16 trainer's scales.  Prints per-parameter and per-layer input-gradient
relative errors.  GPU only; test infrastructure (uses oracle/ via tests/parity_util.py).

    python scripts/grad_error_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import importlib  # noqa: E402

from oracle import ref_model as R  # noqa: E402
from parity_util import grad_errors, report, run_model_pair  # noqa: E402

mm = importlib.import_module("multimodal-s2ut_amd")

cases = [
    ("smoke tiny", R.no_dropout(R.tiny_config(conv_channels=256)), [61, 47], [14, 11], 17),
    ("base 2+1", R.no_dropout(R.base_config(encoder_layers=2, decoder_layers=1)), [120, 97], [37, 29], 37),
]
for name, cfg, L, T, Ti in cases:
    for replay in (False, True):
        for scale in (1.0, 128.0):
            r = run_model_pair(mm, cfg, L, T, img_tokens=Ti, seed=0, scale=scale, replay_relu=replay)
            e = grad_errors(r)
            fc1 = e.get("encoder.transformer_layers.0.fc1.weight")
            print(f"== {name} relu-replay {replay} scale {scale:g}: max grad err {max(e.values()):.3e} "
                  f"enc0.fc1 {fc1:.3e}")
            print(report(r, top=6), flush=True)
