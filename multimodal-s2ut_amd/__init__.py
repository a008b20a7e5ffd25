"""multimodal-s2ut_amd — MI355X-native training path for whxhcj/multimodal-S2UT's
``mm_s2ut_transformer`` (fbank front end -> Conv1d subsampler -> pre-LN speech encoder ->
gated audio/image fusion -> unit decoder -> label-smoothed CE), fp16, data-parallel over RCCL.

Import by path (the directory name is not an identifier):
    pkg = importlib.import_module("multimodal-s2ut_amd")
or use it as a fairseq ``--user-dir`` (fairseq imports the directory by its basename).

Plugin names (same as the reference): task ``multimodal_speech_to_speech``, model/arch
``mm_s2ut_transformer``, criterion ``speech_to_unit`` (aliases ``speech_to_speech``,
``speech_to_unit_v2``).
"""
from . import _lib, data, frontend, generate, kernels, manifest, model, multitask, optim, parallel, plugins, runtime, trainer  # noqa: F401
from .model import MMS2UTModel, default_cfg, param_specs  # noqa: F401
from .plugins import REGISTRY  # noqa: F401

try:  # fairseq --user-dir: register the same names into fairseq's registries
    import fairseq as _fairseq
except ImportError:
    _fairseq = None
if _fairseq is not None:
    from . import fairseq_adapter
    fairseq_adapter.register(_fairseq)

__version__ = "0.1.0"
