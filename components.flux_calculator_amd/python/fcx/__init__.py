"""fcx: host-side Python interface of the MI355X exchange-grid flux engine (libfcx.so).

The compute path is the HIP library only (include/fcx.h); this package binds it with
ctypes, mirrors the reference data model and module names, and generates synthetic
exchange-grid inputs.  Importing it does not touch the GPU.
"""
from . import basic, local_field, synthetic  # noqa: F401
from ._lib import FcxError, LIB_PATH  # noqa: F401

__version__ = "0.1.0"
