"""CPU oracle for the mm_s2ut_transformer hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything in this package, and only as the checker / the timed CPU baseline — never as the thing
measured or shipped.  The product path (``multimodal-s2ut_amd``) never imports it and fails
loudly when its HIP library is missing.

Contents
  ref_model.py  — PyTorch-CPU (fp32/fp64) restatement of the fairseq-resident layers the reference
                  runs on (Conv1dSubsampler, sinusoidal positions, pre-LN encoder/decoder layers,
                  TransformerUnitDecoder, label-smoothed CE, FP16Optimizer+Adam) and of the
                  reference's own fusion block.
  ref_fbank.py  — numpy restatement of torchaudio.compliance.kaldi.fbank (the reference's
                  `_get_torchaudio_fbank` path) + utterance CMVN.
  gen_golden.py — writes tests/golden/fusion_*.npz by running the reference's own fusion code
                  under an import shim (container only).

Parity pinning:
  * fusion block (A7–A9): PINNED — checked against golden vectors produced by the reference itself.
  * encoder / decoder (A3–A5, A10): pinned against transformers' Speech2Text port of fairseq's S2T
    transformer where the architectures coincide (independent implementation; the reference's
    fairseq dependency is absent from the container and unpinned) — otherwise "parity unpinned".
  * fbank (A1): cross-checked against transformers.audio_utils' Kaldi-compatible numpy fbank
    (independent implementation); torchaudio itself is absent — "parity unpinned" w.r.t. torchaudio.
  * LS-CE (A11): closed-form known-answer tests.
"""
