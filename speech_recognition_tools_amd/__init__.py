"""MI355X-native FDLP-spectrogram extractor (drop-in for the FDLP path of
sadhusamik/speech_recognition_tools: src/featgen/computeFDLPSpectrogram.py + features.py).

The compute path is libfdlp_hip.so (hand-written gfx950 HIP kernels behind include/fdlp.h); loading it
fails loudly when the library is missing (there is no fallback).  The names below load lazily, so the
native JOB runner of compute-fdlp-feats can choose the HIP runtime before the library is loaded
(speech_recognition_tools_amd._hip_runtime).  torch.ops.fdlp.spectrogram is registered by importing
speech_recognition_tools_amd.ops: on package import when torch was imported first, otherwise when FdlpPlan
is first touched -- a process that imports torch after this package and wants the op before it creates a
plan imports speech_recognition_tools_amd.ops itself.
"""
import importlib
import sys

_LAZY = {"FdlpPlan": ".plan", "FeatureConfig": ".config", "DEFAULT_SUPPORT_EPS": ".config",
         "PyRandom": ".rng", "NpRandom": ".rng", "FdlpError": "._lib", "lib": "._lib", "q_widen": ".plan"}

__all__ = ["FdlpPlan", "FeatureConfig", "PyRandom", "NpRandom", "FdlpError", "DEFAULT_SUPPORT_EPS"]


def __getattr__(name):
    mod = _LAZY.get(name)
    if mod is None:
        raise AttributeError("module %r has no attribute %r" % (__name__, name))
    return getattr(importlib.import_module(mod, __name__), name)


if "torch" in sys.modules:  # torch users: the library on torch's runtime, the custom op registered
    from . import ops  # noqa: F401,E402
