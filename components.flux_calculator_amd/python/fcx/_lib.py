"""ctypes binding of libfcx.so (include/fcx.h).

The product path is the HIP library: loading fails loudly (FcxError) when it has not been
built; there is no CPU fallback anywhere in this package.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libfcx.so"))
# development A/B of two builds of the same library (e.g. launch-bound experiments); the
# override must still be a libfcx build -- there is no other implementation to fall back to
if os.environ.get("FCX_LIBRARY"):
    LIB_PATH = os.path.abspath(os.environ["FCX_LIBRARY"])

FCX_OK = 0
FCX_MEM_HOST = 0x0
FCX_MEM_DEVICE = 0x1
FCX_ALLOCATED = 0x2
FCX_CORR_CELL_MAJOR = 0
FCX_CORR_MONTH_MAJOR = 1
FCX_PRECISION_F64 = 0
FCX_PRECISION_F32 = 1
FCX_COMM_ID_BYTES = 128

# every symbol declared in include/fcx.h: (name, restype, argtypes)
_c = ctypes
_P = _c.c_void_p
_I = _c.c_int
_I32 = _c.c_int32
_I64 = _c.c_int64
_DP = _c.POINTER(_c.c_double)
SIGNATURES = [
    ("fcx_last_error", _c.c_char_p, []),
    ("fcx_version", _I, []),
    ("fcx_method_from_string", _I, [_c.c_char_p, _c.c_size_t]),
    ("fcx_current_month", _I, [_I32, _I64, _c.POINTER(_I32)]),
    ("fcx_create", _I, [_I, _I, _c.POINTER(_I32), _c.POINTER(_P)]),
    ("fcx_destroy", _I, [_P]),
    ("fcx_set_stream", _I, [_P, _P]),
    ("fcx_set_method", _I, [_P, _I, _I, _I]),
    ("fcx_bind_field", _I, [_P, _I, _I, _I, _P, _I64, _I]),
    ("fcx_set_corrections", _I, [_P, _I, _I32, _P, _I64, _I]),
    ("fcx_set_regrid_matrix", _I, [_P, _I, _I64, _P, _P, _P]),
    ("fcx_set_put_to", _I, [_P, _I, _I, _I, _I]),
    ("fcx_add_average", _I, [_P, _I, _I, _I]),
    ("fcx_set_precision", _I, [_P, _I]),
    ("fcx_commit", _I, [_P]),
    ("fcx_plan_check", _I, [_P]),
    ("fcx_upload", _I, [_P, _I]),
    ("fcx_run", _I, [_P, _I, _I32]),
    ("fcx_download", _I, [_P, _I]),
    ("fcx_step", _I, [_P, _I, _I32]),
    ("fcx_synchronize", _I, [_P]),
    ("fcx_calc_spec_vapor_surface", _I, [_P, _I]),
    ("fcx_calc_flux_mass_evap", _I, [_P, _I32]),
    ("fcx_calc_flux_heat_latent", _I, [_P]),
    ("fcx_calc_flux_heat_sensible", _I, [_P]),
    ("fcx_calc_flux_momentum_east", _I, [_P, _I]),
    ("fcx_calc_flux_momentum_north", _I, [_P, _I]),
    ("fcx_calc_flux_radiation_blackbody", _I, [_P]),
    ("fcx_distribute_shortwave_radiation_flux", _I, [_P]),
    ("fcx_average_across_surface_types", _I, [_P, _I, _I]),
    ("fcx_do_regridding", _I, [_P, _I, _I]),
    ("fcx_device_ptr", _I, [_P, _I, _I, _I, _c.POINTER(_DP)]),
    ("fcx_device_layout", _I, [_P, _c.POINTER(_I64), _c.POINTER(_I64)]),
    ("fcx_last_kernel_ms", _I, [_P, _c.POINTER(_c.c_float)]),
    ("fcx_staging_bytes", _I, [_P, _c.POINTER(_I64)]),
    ("fcx_algorithmic_bytes", _I, [_P, _I, _c.POINTER(_I64)]),
    ("fcx_span_runs", _I, [_P, _I, _c.POINTER(_I32), _c.POINTER(_I32)]),
    ("fcx_zero_copy_bytes", _I, [_P, _c.POINTER(_I64)]),
    ("fcx_run_group", _I, [_P, _I, _I, _I32]),
    ("fcx_pinned_bytes", _I, [_P, _c.POINTER(_I64)]),
    ("fcx_handoff_recoveries", _I, [_P, _c.POINTER(_I64)]),
    ("fcx_host_malloc", _I, [_c.c_size_t, _c.POINTER(_P)]),
    ("fcx_set_atmos_boundaries", _I, [_P, _I32, _I32, _I32]),
    ("fcx_comm_unique_id", _I, [_P]),
    ("fcx_comm_create", _I, [_I, _I, _I, _P, _c.POINTER(_P)]),
    ("fcx_comm_destroy", _I, [_P]),
    ("fcx_comm_allreduce_sum", _I, [_P, _P, _c.c_size_t, _P]),
    ("fcx_set_comm", _I, [_P, _P]),
    ("fcx_atmos_allreduce", _I, [_P, _c.POINTER(_P), _I]),
    ("fcx_host_free", _I, [_P]),
    ("fcx_add_remap", _I, [_P, _I64, _I64, _P, _P, _P, _P]),
    ("fcx_add_remap_field", _I, [_P, _I32, _I, _I, _I, _I, _P, _I]),
    ("fcx_remap_info", _I, [_P, _I32, _c.POINTER(_c.c_double), _c.POINTER(_I32)]),
    ("fcx_set_option", _I, [_P, _I, _I64]),
    ("fcx_set_atmos_map", _I, [_P, _I64, _P, _P]),
    ("fcx_add_atmos_field", _I, [_P, _I, _I, _I, _I, _P, _I]),
    ("fcx_set_atmos_shared", _I, [_P, _P, _I32, _I32, _I32, _I32]),
    ("fcx_atmos_finish", _I, [_P]),
    ("fcx_run_atmos", _I, [_P, _I]),
    ("fcx_device_malloc", _I, [_I, _c.c_size_t, _c.POINTER(_P)]),
    ("fcx_device_free", _I, [_P]),
    ("fcx_memcpy", _I, [_P, _P, _c.c_size_t, _I]),
    ("fcx_last_group_size", _I, [_P, _c.POINTER(_I32)]),
    ("fcx_step_async", _I, [_P, _I, _I32]),
    ("fcx_upload_field", _I, [_P, _I, _I, _I]),
    ("fcx_comm_verify", _I, [_P, _I]),
    ("fcx_set_abort_handler", _I, [_P]),
    ("fcx_abort", _I, [_c.c_char_p]),
]


class FcxError(RuntimeError):
    """Non-zero status of a libfcx entry point (message from fcx_last_error)."""

    def __init__(self, status, message):
        super().__init__(f"fcx status {status}: {message}")
        self.status = status


_lib = None


def load():
    """Load libfcx.  libfcx's DT_NEEDED is the unversioned libamdhip64.so, so it binds to the
    HIP runtime already in the process.  PyTorch-ROCm carries its own runtime
    (torch/lib/libamdhip64.so); when torch is installed it is imported first so that the
    process has exactly one HIP runtime (torch's) and torch tensors, streams and events
    can be handed to libfcx directly.  The GPU itself is not touched here."""
    global _lib
    if _lib is None:
        if not os.environ.get("FCX_NO_TORCH"):  # (measurement tools: a torch-free process, as a
            try:                                 # Fortran host is, binds the system HIP runtime)
                import torch  # noqa: F401
            except ImportError:
                pass
        if not os.path.exists(LIB_PATH):
            raise FcxError(-1, f"{LIB_PATH} is not built (run __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        # an FCX_LIBRARY override (A/B of an older build) may predate some entry points
        _bind(lib, strict=not os.environ.get("FCX_LIBRARY"))
        _lib = lib
    return _lib


def load_path(path):
    """A second libfcx build (A/B measurement tools: engines of two builds in one process
    over the same arrays).  The process's own library is still load()'s."""
    load()
    lib = ctypes.CDLL(os.path.abspath(path))
    _bind(lib, strict=False)
    return lib


def _bind(lib, strict=True):
    for name, res, args in SIGNATURES:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if strict:
                raise
            continue
        fn.restype = res
        fn.argtypes = args


def check(status):
    if status != FCX_OK:
        raise FcxError(status, load().fcx_last_error().decode(errors="replace"))
    return status
