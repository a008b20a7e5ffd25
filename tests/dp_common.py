"""Shared model/batches of the data-parallel equivalence test (tests/test_gpu_dp.py, dp_child.py)."""
from oracle import ref_model as R


def model_cfg(mm):
    return mm.default_cfg(**R.no_dropout(R.tiny_config(conv_channels=256)))


# gradient bucket sizes of the DP test: many small buckets (overlap path) + SURVEY §8e's sweep
BUCKETS_MB = (0.25, 8, 25, 64, 128)

SHAPES =(([120, 90], [30, 22]), ([100, 77, 60], [25, 20, 15]))


def samples(mm):
    return [mm.data.make_sample(L, T, img_tokens=37, img_dim=768, seed=s) for s, (L, T) in enumerate(SHAPES)]


def batches(mm, cfg):
    return [mm.runtime.prepare_batch(s, cfg, "cuda") for s in samples(mm)]
