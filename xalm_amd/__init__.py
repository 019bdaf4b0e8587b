"""xalm_amd — MI355X-native (gfx950) single-batch decode path for Xalm's forward().

Product: libxalm_hip.so (HIP kernels + C ABI, include/xalm_hip.h), the C++ host
(libxalm_host.so, bin/xalm) and this thin Python mirror of Model / InferenceState.
"""
from . import _lib
from ._lib import XhError
from .model import InferenceState, Model
from .xalm_file import XalmFile

__all__ = ["Model", "InferenceState", "XalmFile", "XhError", "_lib"]
