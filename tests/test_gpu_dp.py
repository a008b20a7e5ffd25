"""Data-parallel equivalence on the one GPU: two fresh child processes
(tests/dp_child.py) form a world-2 gloo process group sharing cuda:0, each running the real
Trainer on its own batch.  Checks:
  * the DP-reduced gradient (DDP semantics: each bucket divided by world, then SUM) times world
    equals the single-process gradient of the same two batches accumulated with --update-freq 2
    (relative L2 <= 1e-3);
  * both ranks hold bit-identical gradients, parameters, fp32 masters and optimizer state after 3
    updates, and the cross-rank grad-norm check (fairseq Trainer._check_grad_norms) stays clean;
  * the DP run's parameters after 3 updates match the single-process --update-freq 2 run's.
The children run the default configuration: deferred chunked Adam and the gradient zeroing on
the side stream (the gradient is taken right before the optimizer, Trainer.grad_tap), once per
bucket size in dp_common.BUCKETS_MB; every bucket size must give bit-identical results.
Children are spawned (never exec'd over a GPU process) and bounded by a timeout."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg
from dp_common import BUCKETS_MB, batches, model_cfg

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


@pytest.fixture(scope="module")
def dp_run(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path_factory.mktemp("dp")
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MMS2UT_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dp_child.py"), str(out)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=420)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), logs
    return {mb: [dict(np.load(out / f"rank{r}_b{mb:g}.npz")) for r in range(2)] for mb in BUCKETS_MB}


@pytest.fixture(scope="module")
def single_run():
    mm = pkg()
    cfg = model_cfg(mm)
    model = mm.MMS2UTModel(cfg, device="cuda").init_params(seed=5)
    tr = mm.trainer.Trainer(model, lr=1e-3, world_size=1, init_scale=8.0, warmup_updates=0, update_freq=2)
    assert tr.opt.defer
    taps = []
    tr.grad_tap = lambda g: taps.append(g.clone()) if not taps else None
    bs = batches(mm, cfg)
    out = {}
    for step in range(3):
        tr.train_step(bs)
        if step == 0:
            torch.cuda.synchronize()
            out["grad0"] = taps[0].float().cpu().numpy()
            tr.sync()
            out["ost0"] = tr.opt.ost.cpu().numpy()
    tr.sync()
    torch.cuda.synchronize()
    out["master"] = tr.opt.master.cpu().numpy()
    out["ost"] = tr.opt.ost.cpu().numpy()
    return out


@pytest.mark.parametrize("mb", BUCKETS_MB)
def test_dp_ranks_bit_identical(dp_run, mb):
    r0, r1 = dp_run[mb]
    for k in ("grad0", "params", "master", "ost"):
        assert np.array_equal(r0[k], r1[k]), k
    assert not bool(r0["inconsistent"]) and not bool(r1["inconsistent"])
    K = pkg("kernels")
    assert r0["ost"][K.OST_STEP] == 3 and r0["ost"][K.OST_FATAL] == 0


def test_dp_bucket_size_invariant(dp_run):
    """The same sums whatever the bucket cut: every size gives the 0.25 MB run's bits."""
    ref = dp_run[BUCKETS_MB[0]][0]
    assert int(ref["nbuckets"]) > 1 and int(dp_run[BUCKETS_MB[-1]][0]["nbuckets"]) == 1
    for mb in BUCKETS_MB[1:]:
        for k in ("grad0", "params", "master", "ost"):
            assert np.array_equal(dp_run[mb][0][k], ref[k]), (mb, k)


def test_dp_gradient_equals_accumulated_union(dp_run, single_run):
    K = pkg("kernels")
    dp_run = dp_run[BUCKETS_MB[0]]
    dp = dp_run[0]["grad0"] * 2.0              # DDP average -> sum
    assert _rel(dp, single_run["grad0"]) < 1e-3
    # same multiply factor: world / (scale * sample_size) on the average == 1 / (scale * size) on the sum
    assert np.isclose(dp_run[0]["ost0"][K.OST_MULT], 2.0 * single_run["ost0"][K.OST_MULT], rtol=1e-6)
    assert np.isclose(dp_run[0]["ost0"][K.OST_GNORM], single_run["ost0"][K.OST_GNORM], rtol=1e-3)
    # Adam turns near-zero gradient differences into +-lr steps: compare the masters loosely
    assert _rel(dp_run[0]["master"], single_run["master"]) < 1e-3
    assert dp_run[0]["ost"][K.OST_LOSS_SCALE] == single_run["ost"][K.OST_LOSS_SCALE]
