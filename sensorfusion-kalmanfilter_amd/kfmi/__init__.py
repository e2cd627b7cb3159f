"""kfmi — MI355X-native batched Kalman-filter engine (HIP kernels behind a C ABI).

Import is cheap and never touches the GPU; the shared library is loaded on first use and
its absence raises KFError (there is no CPU fallback).
"""
from ._lib import KFError, KF_ENOTSPD, KF_OK, header_functions, lib  # noqa: F401
from .engine import MODELS, BatchedKF, default_params, device_count  # noqa: F401

__version__ = '0.1.0'
