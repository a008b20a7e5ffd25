"""fairseq drop-in under torch DDP: two fresh child processes
(tests/dp_fairseq_child.py) form a world-2 gloo process group sharing cuda:0 and train the adapter
model wrapped the way fairseq's distributed_fairseq_model wraps it (DDP, bucket_cap_mb 25,
broadcast_buffers False, find_unused_parameters False), each rank on its own batch.  Checks:
  * both ranks hold bit-identical averaged gradients, and every bucket size gives the same bits;
  * the DDP gradient times world equals the single-process gradient of the same two batches
    accumulated with --update-freq 2 (relative L2 <= 1e-3);
  * DDP's bucket all-reduces start while the hand-written backward is still running (the
    adapter hands each parameter group to autograd as soon as it is final) — on the second
    iteration, after DDP rebuilt its buckets in gradient-ready order.
Children are spawned (never exec'd over a GPU process) and bounded by a timeout."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg
from test_gpu_plugins import FUSION_NODROP

pytestmark = pytest.mark.gpu

BUCKETS_MB = (25, 1)     # tests/dp_fairseq_child.py
NODROP = "--dropout 0 --attention-dropout 0 --relu-dropout 0"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


def _spawn(out, mode="tiny"):
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MMS2UT_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dp_fairseq_child.py"), str(out),
                                       str(out / "work"), mode], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    return procs


@pytest.fixture(scope="module")
def ddp_run(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path_factory.mktemp("ddp_fs")
    procs = _spawn(out)
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), logs
    runs = {mb: [dict(np.load(out / f"rank{r}_b{mb}.npz")) for r in range(2)] for mb in BUCKETS_MB}
    runs["unused"] = [dict(np.load(out / f"rank{r}_b25u.npz")) for r in range(2)]
    return runs


@pytest.mark.parametrize("mb", BUCKETS_MB)
def test_ddp_ranks_bit_identical(ddp_run, mb):
    r0, r1 = ddp_run[mb]
    assert np.isfinite(r0["grad"]).all()
    assert np.array_equal(r0["grad"], r1["grad"])


def test_ddp_bucket_size_invariant(ddp_run):
    assert np.array_equal(ddp_run[BUCKETS_MB[0]][0]["grad"], ddp_run[BUCKETS_MB[1]][0]["grad"])


def test_ddp_find_unused_parameters(ddp_run):
    """fairseq --find-unused-parameters: DDP walks the graph from the loss, so the adapter switches
    to the loss-linked gradient bridge (fairseq_adapter._LinkedBridge).  Ranks agree bit
    for bit, and the averaged gradient is the per-group release's bit for bit."""
    r0, r1 = ddp_run["unused"]
    assert np.isfinite(r0["grad"]).all()
    assert np.array_equal(r0["grad"], r1["grad"])
    assert np.array_equal(r0["grad"], ddp_run[BUCKETS_MB[0]][0]["grad"])


def test_ddp_buckets_overlap_backward(ddp_run):
    """Second iteration, 1 MB buckets: most buckets are launched while parameter groups are still
    waiting for the hand-written backward (the tiny model's 12.6 MB of fp16 gradients fill one
    25 MB bucket, which can only fire at the end; the base model's 301 MB fill twelve)."""
    for r in range(2):
        lz = ddp_run[1][r]["launches1"]
        assert len(lz) >= 4, lz
        early = int((lz[:, 1] > 0).sum())
        assert early >= len(lz) // 2, lz
        assert int(lz[-1, 1]) == 0, lz      # the last bucket closes with the last group
        print(f"rank {r} iteration 2 buckets (index, groups pending, elements):", lz.tolist())


def test_ddp_gradient_equals_update_freq_2(ddp_run, monkeypatch, tmp_path):
    import fairseq_stub
    pkg()       # imported before the stub exists: no --user-dir auto-registration (__init__.py)
    fs, regs, args, c, _ = fairseq_stub.dropin_setup(monkeypatch, tmp_path, FUSION_NODROP, extra=NODROP)
    task = fs.tasks.setup_task(args)
    task.load_dataset("train")
    model = task.build_model(args).half()
    crit = regs["criterion"]["speech_to_unit_v2"].build_criterion(args, task)
    batches = task.get_batch_iterator(task.dataset("train"), max_tokens=450, max_positions=task.max_positions())
    net = model.impl.net
    model.train()
    model.zero_grad(set_to_none=True)
    for r in range(2):              # fairseq --update-freq 2: grads accumulate into p.grad
        net.drop.reset(11 + r)
        loss, ss, log = crit(model, fs.utils.apply_half(fs.utils.move_to_cuda(batches[r])))
        loss.backward()
    torch.cuda.synchronize()
    ref = torch.cat([p.grad.float().flatten() for _, p in model.named_parameters()]).cpu().numpy()
    dp = ddp_run[BUCKETS_MB[0]][0]["grad"] * 2.0       # DDP average -> sum
    assert dp.shape == ref.shape
    assert _rel(dp, ref) < 1e-3


# ------------------------------------------------------------------ base size
BASE_ARGS = NODROP + (" --encoder-layers 12 --decoder-layers 6 --encoder-embed-dim 768 --encoder-ffn-embed-dim 3072 "
                      "--encoder-attention-heads 8 --decoder-embed-dim 768 --decoder-ffn-embed-dim 3072 "
                      "--decoder-attention-heads 8")


@pytest.fixture(scope="module")
def ddp_base_run(tmp_path_factory):
    """The base 12 + 6 model (301 MB of fp16 gradients) under fairseq's DDP wrap at world 2, 25 MB
    buckets: both ranks' averaged gradients and bucket launch logs."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path_factory.mktemp("ddp_fs_base")
    procs = _spawn(out, "base")
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), logs
    return [dict(np.load(out / f"rank{r}_b25.npz")) for r in range(2)]


def test_ddp_base_ranks_bit_identical(ddp_base_run):
    r0, r1 = ddp_base_run
    assert r0["grad"].size > 140e6          # ~150 M parameters (301 MB of fp16 gradients)
    assert np.isfinite(r0["grad"]).all()
    assert np.array_equal(r0["grad"], r1["grad"])


def test_ddp_base_buckets_overlap_backward(ddp_base_run):
    """Second iteration: of the ~12 buckets of 25 MB, at least 8 are all-reduced while parameter
    groups are still waiting for the hand-written backward."""
    for r in range(2):
        lz = ddp_base_run[r]["launches1"]
        early = int((lz[:, 1] > 0).sum())
        print(f"rank {r}: {len(lz)} buckets, {early} launched before the last group's release:", lz.tolist())
        assert len(lz) >= 10, lz
        assert early >= 8, lz
        assert int(lz[-1, 1]) == 0, lz


def test_ddp_base_gradient_equals_update_freq_2(ddp_base_run, monkeypatch, tmp_path):
    import fairseq_stub
    pkg()
    fs, regs, args, c, _ = fairseq_stub.dropin_setup(monkeypatch, tmp_path, FUSION_NODROP, extra=BASE_ARGS)
    task = fs.tasks.setup_task(args)
    task.load_dataset("train")
    model = task.build_model(args).half()
    crit = regs["criterion"]["speech_to_unit_v2"].build_criterion(args, task)
    batches = task.get_batch_iterator(task.dataset("train"), max_tokens=450, max_positions=task.max_positions())
    net = model.impl.net
    model.train()
    model.zero_grad(set_to_none=True)
    for r in range(2):
        net.drop.reset(11 + r)
        loss, ss, log = crit(model, fs.utils.apply_half(fs.utils.move_to_cuda(batches[r])))
        loss.backward()
    torch.cuda.synchronize()
    ref = torch.cat([p.grad.float().flatten() for _, p in model.named_parameters()]).cpu().numpy()
    dp = ddp_base_run[0]["grad"] * 2.0
    assert dp.shape == ref.shape
    err = _rel(dp, ref)
    print("base DDP x world vs --update-freq 2: rel L2", err)
    assert err < 1e-3
