"""Python mirror of local_field(0:MAX_SURFACE_TYPES, 3)%var(MAX_VARNAMES)%field(:).

The reference keeps one 1-D REAL(wp) POINTER array per (surface type, grid, variable)
(flux_calculator_basic.F90:86-103, flux_calculator.F90:159) and expresses sharing by
pointer aliasing.  LocalFields does the same: a slot holds an array object, and aliasing is
holding the SAME object in several slots.  Arrays are numpy float64 (host, as Fortran owns
them) or torch CUDA float64 tensors (device-resident use, zero copy); a LocalFields built
with dtype="float32" holds float32 arrays for the fp32 engine (FCX_PRECISION_F32).
"""
import numpy as np

from .basic import IDX, MAX_SURFACE_TYPES, VARNAMES


def data_ptr(a):
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


def is_device(a):
    return not isinstance(a, np.ndarray)


def dtype_name(a):
    """'float64' / 'float32' / ... of a numpy array or torch tensor."""
    return str(a.dtype).replace("torch.", "")


class LocalFields:
    def __init__(self, grid_size, device=None, dtype="float64"):
        if dtype not in ("float64", "float32"):
            raise ValueError(f"dtype {dtype}: float64 or float32")
        self.grid_size = [int(n) for n in grid_size]
        self.device = device  # None: numpy host arrays; else a torch device
        self.dtype = dtype
        self.field = {}  # (s, g, name) -> array
        self.allocated = set()  # (s, g, name) with realarray%allocated = .TRUE.
        self.put_to = {}  # (s, g, name) -> bitmask t=1,u=2,v=4

    # ---- helpers
    def _new(self, n, value=None):
        if self.device is None:
            a = np.empty(n, dtype=self.dtype)
            if value is not None:
                a[:] = value
            return a
        import torch

        a = torch.empty(n, dtype=getattr(torch, self.dtype), device=self.device)
        if value is not None:
            a.fill_(value)
        return a

    def associated(self, s, g, name):
        return (s, g, name) in self.field

    def get(self, s, g, name):
        return self.field.get((s, g, name))

    def __getitem__(self, key):
        return self.field[key]

    # ---- flux_calculator_basic.F90 operations
    def allocate_localvar(self, name, s, g, value=None):
        """basic:288-309 (+ init_localvar basic:313-330 when value is given)."""
        if name not in IDX:
            raise KeyError(f"Could not allocate local variable {name} because flux_calculator "
                           "does not know this variable.")
        a = self._new(self.grid_size[g - 1], value)
        self.field[(s, g, name)] = a
        self.allocated.add((s, g, name))
        return a

    def set_array(self, name, s, g, array, allocated=True):
        """Bind an existing array (e.g. synthetic data) to a slot."""
        self.field[(s, g, name)] = array
        if allocated:
            self.allocated.add((s, g, name))
        else:
            self.allocated.discard((s, g, name))
        return array

    def distribute_input_field(self, name, g, from_s, to_s, num_surface_types):
        """basic:334-358: pointer copies of (from_s, g) into other surface types."""
        src = self.field[(from_s, g, name)]
        for j in range(1, num_surface_types + 1):
            if j == to_s or (j != from_s and to_s == 0):
                self.field[(j, g, name)] = src
                self.allocated.discard((j, g, name))

    def alias(self, name, s, g, from_s=1):
        """'copy' method (prepare:36-38) or uniform output alias (basic:205)."""
        self.field[(s, g, name)] = self.field[(from_s, g, name)]
        self.allocated.discard((s, g, name))

    def slots(self):
        for (s, g, name), a in self.field.items():
            yield s, g, IDX[name], a, ((s, g, name) in self.allocated)

    def to_numpy(self, s, g, name):
        a = self.field[(s, g, name)]
        if isinstance(a, np.ndarray):
            return a
        return a.detach().cpu().numpy()


    def astype(self, dtype):
        """A copy with every array converted to dtype (rounded once), aliases kept."""
        new = LocalFields(self.grid_size, self.device, dtype)
        conv = {}
        for key, a in self.field.items():
            if id(a) not in conv:
                if isinstance(a, np.ndarray):
                    conv[id(a)] = np.ascontiguousarray(a, dtype=dtype)
                else:
                    import torch

                    conv[id(a)] = a.to(getattr(torch, dtype)).contiguous()
            new.field[key] = conv[id(a)]
        new.allocated = set(self.allocated)
        new.put_to = dict(self.put_to)
        return new


def rehome(lf, buf, offset, first_key=None):
    """Move every distinct host array of lf into the flat numpy buffer `buf`, back to back
    from byte `offset` (aliases stay one array); first_key = (s, g, name) goes first.
    Returns the byte offset after the last array.  Tests use it to control which arrays
    share memory pages (fcx page-lock registry)."""
    if offset % 8:
        raise ValueError("offset must be a multiple of 8 bytes")
    order = list(lf.field)
    if first_key is not None:
        order.remove(first_key)
        order.insert(0, first_key)
    moved = {}
    for key in order:
        a = lf.field[key]
        if id(a) not in moved:
            if not isinstance(a, np.ndarray):
                raise TypeError("rehome: host arrays only")
            n = a.shape[0]
            if offset + a.nbytes > buf.nbytes:
                raise ValueError("rehome: buffer too small")
            v = np.frombuffer(buf, dtype=a.dtype, count=n, offset=offset)
            v[:] = a
            moved[id(a)] = (a, v)
            offset += a.nbytes
        lf.field[key] = moved[id(a)][1]
    return offset


__all__ = ["LocalFields", "data_ptr", "dtype_name", "is_device", "rehome", "VARNAMES", "MAX_SURFACE_TYPES"]
