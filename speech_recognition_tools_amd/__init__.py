"""MI355X-native FDLP-spectrogram extractor (drop-in for the FDLP path of
sadhusamik/speech_recognition_tools: src/featgen/computeFDLPSpectrogram.py + features.py).

The compute path is libfdlp_hip.so (hand-written gfx950 HIP kernels behind include/fdlp.h);
importing this package fails loudly when that library is missing.
"""
from ._lib import FdlpError, lib  # noqa: F401
from .plan import DEFAULT_SUPPORT_EPS, FdlpPlan, FeatureConfig  # noqa: F401
from .rng import NpRandom, PyRandom  # noqa: F401
from . import ops  # noqa: F401,E402  (registers torch.ops.fdlp.spectrogram)

__all__ = ["FdlpPlan", "FeatureConfig", "PyRandom", "NpRandom", "FdlpError", "DEFAULT_SUPPORT_EPS"]
