"""gibbssampling_amd — MI355X-native (gfx950) hot path of the Gibbs motif sampler.

Drop-in for the per-iteration loop of Etschbeijer/GibbsSampling
(MotifSampler.findBestMotifIndicesByWithStartPositions, GibbsSampling.fs:935-970):
hand-written HIP kernels behind the C ABI in include/gibbs_hip.h.
"""
from . import bioarray
from ._native import (ArgumentError, ChecksumOverflowError, Context, DeviceError, GibbsError,
                      RouletteOverrunError, load_library)
from .sampler import MotifIndex, MotifSampler, SiteSampler, createMotifIndex

__all__ = [
    "bioarray", "Context", "load_library", "MotifIndex", "MotifSampler", "SiteSampler",
    "createMotifIndex", "GibbsError", "ArgumentError", "RouletteOverrunError",
    "ChecksumOverflowError", "DeviceError",
]
__version__ = "0.1.0"
