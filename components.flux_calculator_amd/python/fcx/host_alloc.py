"""Library-owned page-locked host arrays (fcx_host_malloc / fcx_host_free, include/fcx.h).

A host that allocates its local_field arrays from the library gets the zero-copy step on
small grids (the kernels read and write the arrays in place over the host link; the
latency-optimal form for the Baltic-size grid) and direct DMA on large grids, without the
library registering any memory it does not own.  The Fortran equivalent is
fcx_host_malloc + c_f_pointer.
"""
import ctypes

import numpy as np

from . import _lib


class Arena:
    """Owns fcx_host_malloc blocks; numpy views of them live as long as the arena is open.
    Close (or leave the `with` block) only after every engine using the arrays is closed."""

    def __init__(self):
        self.lib = _lib.load()
        self.blocks = []

    def empty(self, n, dtype="float64"):
        dt = np.dtype(dtype)
        p = ctypes.c_void_p()
        _lib.check(self.lib.fcx_host_malloc(max(int(n), 1) * dt.itemsize, ctypes.byref(p)))
        self.blocks.append(p.value)
        buf = (ctypes.c_char * (max(int(n), 1) * dt.itemsize)).from_address(p.value)
        return np.frombuffer(buf, dtype=dt, count=int(n))

    def adopt(self, lf):
        """Move every distinct host array of a LocalFields into arena memory (aliases kept)."""
        moved = {}
        for key, a in list(lf.field.items()):
            if not isinstance(a, np.ndarray):
                continue
            if id(a) not in moved:
                v = self.empty(a.shape[0], a.dtype)
                v[:] = a
                moved[id(a)] = (a, v)
            lf.field[key] = moved[id(a)][1]
        return lf

    def close(self):
        for p in self.blocks:
            self.lib.fcx_host_free(ctypes.c_void_p(p))
        self.blocks = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


__all__ = ["Arena"]
