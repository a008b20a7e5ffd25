"""mms2ut-train: the canonical fairseq-train command line on the HIP path (see cli.py)."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    sys.exit(importlib.import_module("multimodal-s2ut_amd.cli").main())
