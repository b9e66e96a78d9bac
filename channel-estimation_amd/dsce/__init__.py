"""dsce — MI355X-native doubly-selective MMSE channel-estimation engine.

Host-side mirror of the reference's MATLAB class surfaces (``modulation``,
``channel``, ``estimation``), the experiment setup of
DoublySelectiveChannelEstimation.m (``configs``) and the ctypes binding of the
HIP engine (``engine``, C-ABI in include/dsce.h).
"""
from .configs import Scheme, Setup, build_setup  # noqa: F401

__all__ = ["Scheme", "Setup", "build_setup"]
