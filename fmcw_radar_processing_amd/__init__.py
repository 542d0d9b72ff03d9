"""MI355X-native FMCW radar DSP path (drop-in for radar_processing.m's loop).

Product code only: the HIP kernels live in libfmcw.so (csrc/), reached via the
C-ABI of include/fmcw.h.  The test oracle lives in /oracle and is never
imported from here.
"""
from ._lib import (FMCW_C32H, FMCW_C64, FMCW_PIPE_AUTO, FMCW_PIPE_ONEPASS, FMCW_PIPE_STREAMS, FMCW_PIPE_XCD,  # noqa: F401
                   FmcwError)
from .params import FmcwConfig, calibration, config, derive_params, deployed_device  # noqa: F401

__all__ = ["Engine", "FmcwConfig", "FmcwError", "calibration", "config", "derive_params",
           "deployed_device", "radar_processing"]


def __getattr__(name):
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name == "radar_processing":
        from .radar import radar_processing
        return radar_processing
    raise AttributeError(name)
