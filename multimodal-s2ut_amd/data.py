"""Synthetic Speech-Multi30K-shaped batches + the reference's collater contract.

Collation follows ``MultiModalSpeechToSpeechDataset.collater`` / ``_collate_target``
(mm_s2ut/data/speech_to_speech_dataset.py:344-471): frames zero-padded [B, Tmax, 80] and sorted by
length (descending); targets = unit ids + <eos>, right-padded with <pad>=1; prev_output_tokens =
<eos> moved to the front (fairseq collate_tokens(move_eos_to_beginning=True)); imgs_list =
[stack of [Ti, Di] features] reordered; img_masks_list = [None | stacked bool masks].

Batching follows fairseq ``batch_by_size`` with max_tokens: indices sorted by length, a batch
grows while (n+1) * max_len <= max_tokens (SURVEY.md §8d assumptions: Ts ~ clip(N(400,120),
150, 1000); Tt = round(0.3 Ts) + 1; units uniform in [4, 1004); ViT feats [577, 768] ~ N(0,1)).
"""
import numpy as np
import torch

PAD, EOS = 1, 2


def collate_tokens(values, pad_idx, eos_idx, move_eos_to_beginning=False):
    """fairseq data_utils.collate_tokens (left_pad=False)."""
    size = max(v.size(0) for v in values)
    res = values[0].new(len(values), size).fill_(pad_idx)
    for i, v in enumerate(values):
        dst = res[i][: len(v)]
        if move_eos_to_beginning:
            assert v[-1] == eos_idx
            dst[0] = eos_idx
            dst[1:] = v[:-1]
        else:
            dst.copy_(v)
    return res


def collater(items, pad=PAD, eos=EOS):
    """items: list of dicts {index, source [T, C] float (or n_frames: int when the features are
    computed on the GPU), target [Tt] long (ends with eos), img [Ti, Di] or None, img_mask [Ti]
    bool or None}.  Returns the reference's sample dict (src_tokens None without "source")."""
    if len(items) == 0:
        return {}
    indices = torch.tensor([x["index"] for x in items], dtype=torch.long)
    feats = "source" in items[0]
    n_frames = torch.tensor([x["source"].size(0) if feats else x["n_frames"] for x in items], dtype=torch.long)
    frames = None  # items without "source": the GPU front end produces src_tokens from waveforms
    if feats:
        C = items[0]["source"].size(1)
        frames = torch.zeros(len(items), int(n_frames.max()), C, dtype=torch.float32)
        for i, x in enumerate(items):
            frames[i, : x["source"].size(0)] = x["source"]
    n_frames, order = n_frames.sort(descending=True)
    indices = indices.index_select(0, order)
    if feats:
        frames = frames.index_select(0, order)
    targets = [x["target"] for x in items]
    target = collate_tokens(targets, pad, eos).index_select(0, order)
    prev = collate_tokens(targets, pad, eos, move_eos_to_beginning=True).index_select(0, order)
    target_lengths = torch.tensor([t.size(0) for t in targets], dtype=torch.long).index_select(0, order)
    ntokens = sum(t.size(0) for t in targets)
    imgs_list, img_masks_list = [], []
    if items[0].get("img") is not None:
        imgs_list = [torch.stack([x["img"] for x in items]).index_select(0, order)]
        if items[0].get("img_mask") is not None:
            img_masks_list = [torch.stack([x["img_mask"] for x in items]).index_select(0, order)]
        else:
            img_masks_list = [None]
    _o = order.tolist()
    net_input = {
        "src_tokens": frames, "src_lengths": n_frames, "prev_output_tokens": prev,
        "tgt_speaker": None,
        "src_audio_path": [items[i].get("audio_path") for i in _o],
        "img_path": [None for _ in _o], "img_tensor": [None for _ in _o],
        "imgs_list": imgs_list, "img_masks_list": img_masks_list,
    }
    return {"id": indices, "net_input": net_input, "speaker": None, "target": target,
            "target_lengths": target_lengths, "ntokens": ntokens, "nsentences": len(items)}


def synth_lengths(n, rng, mean=400.0, std=120.0, lo=150, hi=1000):
    return np.clip(np.round(rng.normal(mean, std, n)), lo, hi).astype(np.int64)


def batch_by_size(lengths, max_tokens, order=None):
    """fairseq batch_by_size (num_tokens_fn = src length, required_batch_size_multiple 1): walk the
    indices in ``order`` (default: length-sorted) and close a batch when (n+1)*max_len > max_tokens."""
    if order is None:
        order = np.argsort(lengths, kind="stable")
    batches, cur, cur_max = [], [], 0
    for i in order:
        L = int(lengths[i])
        new_max = max(cur_max, L)
        if cur and (len(cur) + 1) * new_max > max_tokens:
            batches.append(cur)
            cur, new_max = [], L
        cur.append(int(i))
        cur_max = new_max
    if cur:
        batches.append(cur)
    return batches


def padded_cost(batch_lengths):
    """Cost proxy of one batch for DP balancing: padded source frames B * Ts_max (what the GEMMs and
    the fbank front end scale with) times 1 + Ts_max / 18432, the self-attention share of an encoder
    layer at the base dims (4 Te^2 d over Te (8d^2 + 4dF) with Te = Ts / 4)."""
    if not len(batch_lengths):
        return 0.0
    t = max(batch_lengths)
    return len(batch_lengths) * t * (1.0 + t / 18432.0)


def deal_batches(costs, world, seed, epoch=1, balanced=True):
    """Assign batches to DP ranks for one epoch -> list (per rank) of batch indices, equal lengths.

    balanced=False: fairseq's ShardedIterator — shuffle with (seed, epoch), drop the tail that does
    not fill every rank, rank r takes positions r, r+world, ...
    balanced=True (token-balanced sharding): sort the batches by ``costs``, cut the
    sorted list into groups of ``world`` neighbours (similar padded cost), shuffle the group order
    with (seed, epoch) and give rank r the r-th member of every group, so the ranks of one update
    step run batches of near-equal cost and no rank waits on a long-tail batch of another.  The
    dropped tail is the ``len % world`` cheapest batches."""
    n = len(costs)
    rs = np.random.RandomState((seed + epoch) % 2 ** 32)
    if not balanced or world == 1:
        order = rs.permutation(n).tolist()
        order = order[: n // world * world]
        return [order[r::world] for r in range(world)]
    srt = np.argsort(np.asarray(costs, dtype=np.float64), kind="stable")[n % world:]
    groups = srt.reshape(-1, world) if len(srt) else np.zeros((0, world), np.int64)
    groups = groups[rs.permutation(len(groups))]
    return [groups[:, r].tolist() for r in range(world)]


class SyntheticSpeechMulti30K:
    """Deterministic synthetic corpus: per-utterance fbank-like features (or waveforms for the
    GPU front end), unit targets and ViT/DETR image features."""

    def __init__(self, n_utts=2000, seed=1, feat_dim=80, vocab=1004, img_tokens=577, img_dim=768,
                 with_images=True, img_mask=False, len_mean=400.0, len_std=120.0, len_lo=150,
                 len_hi=1000):
        self.rng = np.random.default_rng(seed)
        self.n = n_utts
        self.lengths = synth_lengths(n_utts, self.rng, len_mean, len_std, len_lo, len_hi)
        self.tgt_lengths = np.round(0.3 * self.lengths).astype(np.int64) + 1
        self.feat_dim, self.vocab = feat_dim, vocab
        self.img_tokens, self.img_dim = img_tokens, img_dim
        self.with_images, self.img_mask = with_images, img_mask
        self.seed = seed

    def item(self, i, features=True):
        r = np.random.default_rng((self.seed, i))
        T = int(self.lengths[i])
        it = {"index": i, "audio_path": f"{i + 1}.wav"}
        if features:
            it["source"] = torch.from_numpy(r.standard_normal((T, self.feat_dim)).astype(np.float32))
        else:
            it["n_frames"] = T
        nt = int(self.tgt_lengths[i])
        units = r.integers(4, self.vocab, nt - 1)
        it["target"] = torch.from_numpy(np.concatenate([units, [EOS]]).astype(np.int64))
        if self.with_images:
            it["img"] = torch.from_numpy(r.standard_normal((self.img_tokens, self.img_dim)).astype(np.float32))
            if self.img_mask:
                k = int(r.integers(self.img_tokens // 2, self.img_tokens + 1))
                m = torch.zeros(self.img_tokens, dtype=torch.bool)
                m[k:] = True
                it["img_mask"] = m
        return it

    def batches(self, max_tokens=40000):
        return batch_by_size(self.lengths, max_tokens)

    def sample(self, indices):
        return collater([self.item(i) for i in indices])


def make_sample(lengths, tgt_lengths, feat_dim=80, vocab=1004, img_tokens=577, img_dim=768,
                with_images=True, img_mask=False, seed=0):
    """Explicit small batch (tests): one item per given source length."""
    r = np.random.default_rng(seed)
    items = []
    for i, (T, nt) in enumerate(zip(lengths, tgt_lengths)):
        it = {"index": i, "source": torch.from_numpy(r.standard_normal((T, feat_dim)).astype(np.float32))}
        units = r.integers(4, vocab, nt - 1)
        it["target"] = torch.from_numpy(np.concatenate([units, [EOS]]).astype(np.int64))
        if with_images:
            it["img"] = torch.from_numpy(r.standard_normal((img_tokens, img_dim)).astype(np.float32))
            if img_mask:
                k = int(r.integers(img_tokens // 2, img_tokens + 1))
                m = torch.zeros(img_tokens, dtype=torch.bool)
                m[k:] = True
                it["img_mask"] = m
        items.append(it)
    return collater(items)
