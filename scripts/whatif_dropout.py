"""What-if bound on the dropout-hash cost in the step: run bench.py with chosen dropout rates forced
to 0 (activation / residual / attention), everything else unchanged.  Not a valid bench line (the
workload changes); it only bounds what moving the keep-mask hashing off the critical path could save.
usage: WHATIF="activation_dropout,dropout" python scripts/whatif_dropout.py [bench.py args]"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mm = importlib.import_module("multimodal-s2ut_amd")
zero = [k for k in os.environ.get("WHATIF", "").split(",") if k]
_orig = mm.default_cfg


def patched(**kw):
    cfg = _orig(**kw)
    for k in zero:
        assert k in cfg, k
        cfg[k] = 0.0
    return cfg


mm.default_cfg = patched
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
bench = importlib.import_module("bench")
bench.main()
