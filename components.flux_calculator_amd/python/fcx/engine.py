"""Engine: one libfcx engine bound to a LocalFields (one rank, one GPU)."""
import ctypes

import numpy as np

from . import _lib
from .basic import FLUX_ID, IDX, METHOD_ID, PHASE_ALL, PHASE_EARLY, PHASE_NORMAL
from .local_field import LocalFields, data_ptr, dtype_name, is_device


class Engine:
    """Binds every slot of a LocalFields to a new libfcx engine and commits it.

    methods: {which_table_name: [method string per surface type 1..T]}
    corrections: None or (init_date, array) with array shaped like the Fortran
        corrections(1, 12, grid_size(1)) -> numpy [n][12] (cell-major) or [12][n].
    averages: iterable of (phase, grid, name) type-0 outputs averaged before their put.
    """

    def __init__(self, lf: LocalFields, num_surface_types, methods, corrections=None,
                 averages=(), regrid=None, device=0, stream=None, atmos=None, options=None, remaps=None,
                 lib=None, commit=True):
        """atmos: exchange -> atmosphere accumulation, dict with
             local   : fcx.parallel.LocalAtmos of this rank
             fields  : [(phase, surface_type, grid, name, out_array[n_atmos])]
             shared  : optional (device_buffer[n_boundaries * stride], stride)
             own_boundaries : optional True: the engine allocates its boundary slots
                       (fcx_set_atmos_boundaries) from local.n_boundaries/left/right
             comm    : optional fcx.comm.Comm: the engine completes its boundary slots
                       itself after every accumulation (fcx_set_comm)
        remaps: exchange -> model remaps, each {"n_dst", "src", "dst", "w" (0-based links),
                 "fields": [(phase, surface_type, grid, name, out_array[n_dst])]}
        options: {name: value} for fcx_set_option.
        lib: another libfcx build from _lib.load_path (A/B measurement tools only).
        commit=False: bind only (no GPU touched); plan_check() then audits the plans on the host."""
        self.lib = lib if lib is not None else _lib.load()
        self.lf = lf
        self.T = int(num_surface_types)
        self.methods = {k: list(v) for k, v in methods.items()}
        self._keep = []
        h = ctypes.c_void_p()
        gs = (ctypes.c_int32 * 3)(*lf.grid_size)
        _lib.check(self.lib.fcx_create(device, self.T, gs, ctypes.byref(h)))
        self.h = h
        try:
            if stream is not None:
                _lib.check(self.lib.fcx_set_stream(h, ctypes.c_void_p(stream)))
            dtype = getattr(lf, "dtype", "float64")
            self.precision = dtype
            _lib.check(self.lib.fcx_set_precision(
                h, _lib.FCX_PRECISION_F32 if dtype == "float32" else _lib.FCX_PRECISION_F64))
            for table, per_type in self.methods.items():
                for s, m in enumerate(per_type[: self.T], start=1):
                    mid = METHOD_ID[m.rstrip()] if isinstance(m, str) else int(m)
                    _lib.check(self.lib.fcx_set_method(h, FLUX_ID[table], s, mid))
            for s, g, var, a, alloc in lf.slots():
                flags = (_lib.FCX_MEM_DEVICE if is_device(a) else _lib.FCX_MEM_HOST)
                if alloc:
                    flags |= _lib.FCX_ALLOCATED
                if dtype_name(a) != dtype:
                    raise TypeError(f"slot {(s, g, var)}: {dtype_name(a)} array in a {dtype} LocalFields")
                n = a.shape[0]
                _lib.check(self.lib.fcx_bind_field(h, s, g, var, ctypes.c_void_p(data_ptr(a)), n, flags))
            if corrections is not None:
                init_date, corr = corrections
                corr = np.ascontiguousarray(corr, dtype=np.float64)
                layout = _lib.FCX_CORR_CELL_MAJOR if corr.shape[-1] == 12 else _lib.FCX_CORR_MONTH_MAJOR
                self._keep.append(corr)
                _lib.check(self.lib.fcx_set_corrections(h, 1, int(init_date), ctypes.c_void_p(corr.ctypes.data),
                                                        lf.grid_size[0], layout))
            if regrid:
                for which, (src, dst, w) in regrid.get("matrices", {}).items():
                    src = np.ascontiguousarray(src, dtype=np.int32)
                    dst = np.ascontiguousarray(dst, dtype=np.int32)
                    w = np.ascontiguousarray(w, dtype=np.float64)
                    self._keep += [src, dst, w]
                    _lib.check(self.lib.fcx_set_regrid_matrix(
                        h, which, src.shape[0], ctypes.c_void_p(src.ctypes.data),
                        ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(w.ctypes.data)))
            for (s, g, name), mask in lf.put_to.items():
                _lib.check(self.lib.fcx_set_put_to(h, s, g, IDX[name], mask))
            for phase, g, name in averages:
                _lib.check(self.lib.fcx_add_average(h, phase, g, IDX[name]))
            if atmos is not None:
                la = atmos["local"]
                idx = np.ascontiguousarray(la.atmos_index, dtype=np.int32)
                w = np.ascontiguousarray(la.weight, dtype=np.float64)
                self._keep += [idx, w]
                _lib.check(self.lib.fcx_set_atmos_map(h, la.n_atmos, ctypes.c_void_p(idx.ctypes.data),
                                                      ctypes.c_void_p(w.ctypes.data)))
                for phase, s, g, name, out in atmos["fields"]:
                    if dtype_name(out) != dtype:
                        raise TypeError(f"atmosphere output {name}: {dtype_name(out)} array in a {dtype} engine")
                    flags = _lib.FCX_MEM_DEVICE if is_device(out) else _lib.FCX_MEM_HOST
                    self._keep.append(out)
                    _lib.check(self.lib.fcx_add_atmos_field(h, phase, s, g, IDX[name],
                                                            ctypes.c_void_p(data_ptr(out)), flags))
                if atmos.get("shared") is not None:
                    buf, stride = atmos["shared"]
                    self._keep.append(buf)
                    _lib.check(self.lib.fcx_set_atmos_shared(h, ctypes.c_void_p(data_ptr(buf)), la.n_boundaries,
                                                             stride, la.left, la.right))
                elif atmos.get("own_boundaries"):
                    _lib.check(self.lib.fcx_set_atmos_boundaries(h, la.n_boundaries, la.left, la.right))
                if atmos.get("comm") is not None:
                    self._keep.append(atmos["comm"])
                    _lib.check(self.lib.fcx_set_comm(h, atmos["comm"].h))
            for rm in remaps or ():
                src = np.ascontiguousarray(rm["src"], dtype=np.int32)
                dst = np.ascontiguousarray(rm["dst"], dtype=np.int32)
                w = np.ascontiguousarray(rm["w"], dtype=np.float64)
                self._keep += [src, dst, w]
                rid = ctypes.c_int32()
                _lib.check(self.lib.fcx_add_remap(h, int(rm["n_dst"]), src.shape[0], ctypes.c_void_p(src.ctypes.data),
                                                  ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(w.ctypes.data),
                                                  ctypes.byref(rid)))
                for phase, s, g, name, out in rm["fields"]:
                    if dtype_name(out) != dtype:
                        raise TypeError(f"remap output {name}: {dtype_name(out)} array in a {dtype} engine")
                    flags = _lib.FCX_MEM_DEVICE if is_device(out) else _lib.FCX_MEM_HOST
                    self._keep.append(out)
                    _lib.check(self.lib.fcx_add_remap_field(h, rid.value, phase, s, g, IDX[name],
                                                            ctypes.c_void_p(data_ptr(out)), flags))
            for name, value in (options or {}).items():
                _lib.check(self.lib.fcx_set_option(h, self._option_id(name), int(value)))
            if commit:
                _lib.check(self.lib.fcx_commit(h))
        except Exception:
            self.lib.fcx_destroy(h)
            self.h = None
            raise

    def plan_check(self):
        """fcx_plan_check: every launch plan built on the host and audited (before commit)."""
        _lib.check(self.lib.fcx_plan_check(self.h))

    def commit(self):
        _lib.check(self.lib.fcx_commit(self.h))

    # ---- fused path
    def upload(self, phase=PHASE_ALL):
        _lib.check(self.lib.fcx_upload(self.h, phase))

    def run(self, phase=PHASE_ALL, current_step_time=0):
        _lib.check(self.lib.fcx_run(self.h, phase, int(current_step_time)))

    def download(self, phase=PHASE_ALL):
        _lib.check(self.lib.fcx_download(self.h, phase))

    def step(self, phase=PHASE_ALL, current_step_time=0):
        _lib.check(self.lib.fcx_step(self.h, phase, int(current_step_time)))

    def step_async(self, phase=PHASE_ALL, current_step_time=0):
        """fcx_step_async: the step queued; the host arrays hold the outputs after synchronize()."""
        _lib.check(self.lib.fcx_step_async(self.h, phase, int(current_step_time)))

    def upload_field(self, surface_type, grid, name):
        """fcx_upload_field: one input field handed over (staged by the engine's upload thread)."""
        _lib.check(self.lib.fcx_upload_field(self.h, int(surface_type), int(grid), IDX[name]))

    def set_stream(self, stream):
        """fcx_set_stream: launch on this HIP stream (a raw hipStream_t, e.g. a torch
        stream's .cuda_stream) from now on, e.g. a capturing stream for a HIP graph."""
        _lib.check(self.lib.fcx_set_stream(self.h, ctypes.c_void_p(stream)))

    def do_regridding(self, name, surface_type=0):
        """do_regridding (basic:463-522) of one variable, host arrays in and out."""
        _lib.check(self.lib.fcx_do_regridding(self.h, IDX[name], int(surface_type)))

    def synchronize(self):
        _lib.check(self.lib.fcx_synchronize(self.h))

    def last_kernel_ms(self):
        ms = ctypes.c_float()
        _lib.check(self.lib.fcx_last_kernel_ms(self.h, ctypes.byref(ms)))
        return ms.value

    def algorithmic_bytes(self, phase=PHASE_ALL):
        b = ctypes.c_int64()
        _lib.check(self.lib.fcx_algorithmic_bytes(self.h, phase, ctypes.byref(b)))
        return b.value

    def staging_bytes(self):
        """bytes of the page-locked staging arena of caller heap arrays (fcx_staging_bytes)"""
        b = ctypes.c_int64()
        _lib.check(self.lib.fcx_staging_bytes(self.h, ctypes.byref(b)))
        return b.value

    def zero_copy_bytes(self):
        """bytes of host arrays the kernels use in place (fcx_zero_copy_bytes)"""
        b = ctypes.c_int64()
        _lib.check(self.lib.fcx_zero_copy_bytes(self.h, ctypes.byref(b)))
        return b.value

    def span_runs(self, phase=PHASE_ALL):
        """(uploads, downloads) one step of the phase makes of the fcx_host_malloc arrays with
        the span transport (fcx_span_runs)"""
        a, b = ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self.lib.fcx_span_runs(self.h, phase, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def zero_copy_active(self):
        return self.zero_copy_bytes() > 0

    OPTIONS = {"cells_per_thread": 1, "max_blocks": 2, "nontemporal": 3, "specialize": 4,
               "atmos_in_run": 5, "pipeline_chunks": 7, "pipeline_min_chunk": 8, "zero_copy": 9,
               "timing": 10, "tiled_layout": 11, "remap_pack": 13, "host_staging": 15, "host_threads": 16,
               "atmos_halo": 17, "deferred_scatter": 18, "lib_spans": 19}

    def run_atmos(self, phase=PHASE_ALL):
        _lib.check(self.lib.fcx_run_atmos(self.h, phase))

    def atmos_finish(self):
        """After the all-reduce of the shared boundary buffer (fcx_atmos_finish)."""
        _lib.check(self.lib.fcx_atmos_finish(self.h))

    def remap_info(self, remap_id=0):
        """(scatter, packed) of a remap (fcx_remap_info): packed 0 = gather from the arrays,
        1 = packing pass, 2 = records written by the last run's flux launch."""
        sc, pk = ctypes.c_double(), ctypes.c_int32()
        _lib.check(self.lib.fcx_remap_info(self.h, remap_id, ctypes.byref(sc), ctypes.byref(pk)))
        return sc.value, pk.value

    @classmethod
    def _option_id(cls, name):
        """an OPTIONS name, or a raw enum fcx_option value (measurement builds' extra knobs)"""
        if isinstance(name, int) or (isinstance(name, str) and name.isdigit()):
            return int(name)
        return cls.OPTIONS[name]

    def set_option(self, name, value):
        _lib.check(self.lib.fcx_set_option(self.h, self._option_id(name), int(value)))

    def device_ptr(self, s, g, name):
        p = ctypes.POINTER(ctypes.c_double)()
        _lib.check(self.lib.fcx_device_ptr(self.h, s, g, IDX[name], ctypes.byref(p)))
        return ctypes.cast(p, ctypes.c_void_p).value

    def device_layout(self):
        """(tile, tile_stride) of the engine-owned mirrors: cell j of a device buffer is at
        element (j // tile) * tile_stride + j % tile (fcx_device_layout)."""
        tile, stride = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.fcx_device_layout(self.h, ctypes.byref(tile), ctypes.byref(stride)))
        return tile.value, stride.value

    def last_group_size(self):
        """Engines in the merged launch of this engine's last fcx_run_group (0: ran as fcx_run)."""
        m = ctypes.c_int32()
        _lib.check(self.lib.fcx_last_group_size(self.h, ctypes.byref(m)))
        return m.value

    def close(self):
        if self.h is not None:
            self.lib.fcx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_group(engines, phase=PHASE_ALL, current_step_time=0):
    """fcx_run of every engine, the fused T = 1 flux passes of the same shape as ONE launch
    (fcx_run_group): the same results as Engine.run of each."""
    if not engines:
        return
    lib = engines[0].lib
    arr = (ctypes.c_void_p * len(engines))(*[e.h.value for e in engines])
    _lib.check(lib.fcx_run_group(arr, len(engines), phase, int(current_step_time)))


def current_month(init_date, seconds):
    """datetime_helpers.get_current_date(...)['current_month'] via libfcx."""
    lib = _lib.load()
    m = ctypes.c_int32()
    _lib.check(lib.fcx_current_month(int(init_date), int(seconds), ctypes.byref(m)))
    return m.value


__all__ = ["Engine", "run_group", "current_month", "PHASE_EARLY", "PHASE_NORMAL", "PHASE_ALL"]
