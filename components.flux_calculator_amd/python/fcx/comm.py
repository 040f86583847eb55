"""The one collective of the flux path through libfcx (fcx_comm_*, include/fcx.h): an RCCL
communicator per rank, one all-reduce (sum, fp64) of the atmosphere boundary slots per
coupling step (flux_calculator.F90:1015, create_namcouple.F90:92-98).

The unique id travels between the ranks through whatever the host already has: MPI_Bcast
in the Fortran host; here torch.distributed (any backend) or a callable.
"""
import ctypes

from . import _lib


def unique_id():
    """FCX_COMM_ID_BYTES bytes from ncclGetUniqueId (rank 0)."""
    lib = _lib.load()
    buf = (ctypes.c_char * _lib.FCX_COMM_ID_BYTES)()
    _lib.check(lib.fcx_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return bytes(buf)


class Comm:
    def __init__(self, device, nranks, rank, uid):
        if len(uid) != _lib.FCX_COMM_ID_BYTES:
            raise ValueError("unique id must be FCX_COMM_ID_BYTES bytes")
        self.lib = _lib.load()
        self.nranks, self.rank = int(nranks), int(rank)
        buf = (ctypes.c_char * _lib.FCX_COMM_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        _lib.check(self.lib.fcx_comm_create(int(device), self.nranks, self.rank, ctypes.cast(buf, ctypes.c_void_p),
                                            ctypes.byref(h)))
        self.h = h

    @classmethod
    def from_torch(cls, device):
        """Every rank of the default torch.distributed group: rank 0's id broadcast."""
        import torch
        import torch.distributed as dist

        world, rank = dist.get_world_size(), dist.get_rank()
        backend = dist.get_backend()
        dev = torch.device("cuda", device) if backend == "nccl" else torch.device("cpu")
        t = torch.zeros(_lib.FCX_COMM_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            t.copy_(torch.frombuffer(bytearray(unique_id()), dtype=torch.uint8))
        dist.broadcast(t, 0)
        return cls(device, world, rank, bytes(t.cpu().numpy().tobytes()))

    def allreduce_sum(self, tensor, stream):
        """In-place sum of a contiguous float64 device tensor on a HIP stream (raw handle)."""
        _lib.check(self.lib.fcx_comm_allreduce_sum(self.h, ctypes.c_void_p(tensor.data_ptr()), tensor.numel(),
                                                   ctypes.c_void_p(stream)))

    def atmos_allreduce(self, engines):
        """ONE all-reduce of the boundary slots of this rank's engines, then their finish."""
        arr = (ctypes.c_void_p * len(engines))(*[e.h.value for e in engines])
        _lib.check(self.lib.fcx_atmos_allreduce(self.h, arr, len(engines)))

    def verify(self, every_exchange=True):
        """fcx_comm_verify: the signature agreement before every exchange (hosts that change
        their engine lists at run time) or only before the first of each signature."""
        _lib.check(self.lib.fcx_comm_verify(self.h, int(bool(every_exchange))))

    def close(self):
        if getattr(self, "h", None) is not None:
            self.lib.fcx_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["Comm", "unique_id"]
