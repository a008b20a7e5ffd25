"""BASELINE configs[2] (the base model, data-parallel) rehearsed at world 2 on the one GPU: the driver's
own N > 1 command path — `bench.py --gpus 2` launches its two ranks through torch.distributed.run
(a child process), here over gloo with both ranks on device 0 (parallel.init_from_env maps ranks
past the visible devices onto them when MMS2UT_DIST_BACKEND=gloo).  Full base size, max-tokens
40000, every rank its own corpus at the same length quantile (weak scaling).  Checks at two
gradient bucket sizes (25 / 64 MB): the JSON line reports n_gpus 2 / dp2, the ranks'
fp32 masters are identical, no step was flagged inconsistent by the cross-rank grad-norm check,
and the master checksum does not depend on the bucket cut (the all-reduced sums are the same).
RCCL over xGMI needs one GPU per rank and is exercised only by the driver's 8-GPU runs."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(bucket_mb):
    env = dict(os.environ, MMS2UT_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-gemm-timing", "--bucket-mb", str(bucket_mb)]
    p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=420)
    out = p.stdout.decode(errors="replace")
    assert p.returncode == 0, out[-3000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


@pytest.fixture(scope="module")
def runs():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return {mb: _run(mb) for mb in (25, 64)}


@pytest.mark.parametrize("mb", (25, 64))
def test_bench_dp2_line(runs, mb):
    r = runs[mb]
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["scaling"] == "weak"
    assert r["value"] > 0 and r["ms_per_step"] > 0
    assert r["config"]["model"] == "mm_s2ut_transformer" and r["config"]["max_tokens"] == 40000
    opt = r["optimizer"]
    assert opt["ranks_identical"] and not opt["inconsistent"] and not opt["fatal"]


def test_bench_dp2_bucket_invariant(runs):
    assert runs[25]["optimizer"]["master_checksum"] == runs[64]["optimizer"]["master_checksum"]
