"""The C ABI library: loads without a GPU, exports every symbol include/fcx.h declares,
and its host-side logic (method strings, binding validation, regrid links) behaves like
the reference's prepare step.  No compute call is made here."""
import ctypes
import os
import re

import numpy as np
import pytest

from fcx import _lib
from fcx.engine import Engine
from fcx.synthetic import build_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fcx.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\s*\*|int)\s*(fcx_\w+)\s*\(", text, re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert len(syms) >= 35
    for must in ("fcx_create", "fcx_commit", "fcx_run", "fcx_calc_flux_mass_evap",
                 "fcx_average_across_surface_types", "fcx_do_regridding", "fcx_last_error"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(declared_symbols()) == bound, set(declared_symbols()) ^ bound


def test_fortran_module_binds_every_declared_symbol():
    """fortran/fcx_c_api.F90 carries one BIND(C) interface per entry point of include/fcx.h
    (a Fortran host reaches the whole ABI), and nothing the header no longer declares."""
    f90 = open(os.path.join(ROOT, "components.flux_calculator_amd", "fortran", "fcx_c_api.F90")).read()
    bound = set(re.findall(r"BIND\(C,\s*name='(fcx_\w+)'\)", f90))
    assert bound == set(declared_symbols()), set(declared_symbols()) ^ bound


def test_library_is_gfx950_only_and_unversioned_hip():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"libamdhip64.so.7\0" not in data  # DT_NEEDED rewritten (tools/unversion_needed.py)


@pytest.mark.parametrize("s,expect", [("CCLM", 3), ("CCLM" + " " * 16, 3), ("MOM5", 4), ("RCO ", 5),
                                      ("water", 6), ("ice", 7), ("StBo", 8), ("none", 0), ("zero", 1),
                                      ("copy", 2), ("cclm", -1), ("", -1), ("StBo2", -1)])
def test_method_from_string_trims_like_fortran(s, expect):
    lib = _lib.load()
    b = s.encode()
    assert lib.fcx_method_from_string(b, len(b)) == expect


def test_create_and_validate_without_gpu_missing_input():
    """prepare_flux_mass_evap: CCLM lacking QATM -> error naming the field, before any HIP call."""
    case = build_case("CCLM", n=64, T=1)
    for g in (1, 2, 3):
        case.lf.field.pop((1, g, "QATM"), None)
        case.lf.field.pop((0, g, "QATM"), None)
    with pytest.raises(_lib.FcxError) as ei:
        Engine(case.lf, 1, case.methods)
    assert ei.value.status == 5 and "QATM" in str(ei.value) and "MEVA" in str(ei.value)


def test_unknown_method_rejected():
    case = build_case("CCLM", n=64, T=1)
    bad = dict(case.methods)
    bad["which_flux_heat_latent"] = ["CCLM"]  # not a latent-heat method (prepare:139-142)
    with pytest.raises(_lib.FcxError) as ei:
        Engine(case.lf, 1, bad)
    assert "HLAT" in str(ei.value)


def test_short_array_rejected():
    lib = _lib.load()
    h = ctypes.c_void_p()
    gs = (ctypes.c_int32 * 3)(100, 100, 100)
    _lib.check(lib.fcx_create(0, 1, gs, ctypes.byref(h)))
    a = np.zeros(50)
    st = lib.fcx_bind_field(h, 1, 1, 11, ctypes.c_void_p(a.ctypes.data), 50, 0)
    assert st == 1 and b"shorter than grid_size" in lib.fcx_last_error()
    lib.fcx_destroy(h)


def test_regrid_links_outside_local_grid_rejected():
    """read_regridding_matrix aborts when links leave the task's range (io:183-191)."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    gs = (ctypes.c_int32 * 3)(10, 8, 8)
    _lib.check(lib.fcx_create(0, 1, gs, ctypes.byref(h)))
    src = np.array([1, 11], dtype=np.int32)  # 11 > grid_size(t)
    dst = np.array([1, 2], dtype=np.int32)
    w = np.ones(2)
    st = lib.fcx_set_regrid_matrix(h, 2, 2, ctypes.c_void_p(src.ctypes.data),
                                   ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(w.ctypes.data))
    assert st == 1 and b"outside the local grids" in lib.fcx_last_error()
    lib.fcx_destroy(h)


def test_engine_calls_before_commit_fail_cleanly():
    lib = _lib.load()
    h = ctypes.c_void_p()
    gs = (ctypes.c_int32 * 3)(10, 10, 10)
    _lib.check(lib.fcx_create(0, 1, gs, ctypes.byref(h)))
    assert lib.fcx_run(h, 3, 0) == 2  # FCX_E_STATE
    assert b"fcx_commit" in lib.fcx_last_error()
    assert lib.fcx_create(0, 11, gs, ctypes.byref(h)) == 1  # > MAX_SURFACE_TYPES
    lib.fcx_destroy(h)


def test_tiled_layout_option_and_query_before_commit():
    """FCX_OPT_TILED_LAYOUT (11) is set before fcx_commit; the layout is only known after it."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    gs = (ctypes.c_int32 * 3)(10, 10, 10)
    _lib.check(lib.fcx_create(0, 1, gs, ctypes.byref(h)))
    _lib.check(lib.fcx_set_option(h, 11, 0))
    _lib.check(lib.fcx_set_option(h, 11, 1))
    tile, stride = ctypes.c_int64(), ctypes.c_int64()
    assert lib.fcx_device_layout(h, ctypes.byref(tile), ctypes.byref(stride)) == 2  # FCX_E_STATE
    lib.fcx_destroy(h)


def test_fp32_engine_takes_fp32_outputs_only():
    """The fp32 engine's atmosphere and remap outputs are float arrays (fcx.h
    fcx_set_precision): a float64 output is refused before any HIP call."""
    from fcx.parallel import local_atmos, synthetic_atmos_map
    from fcx.synthetic import as_dtype

    c32 = as_dtype(build_case("CCLM", n=64, T=1), "float32")
    amap = synthetic_atmos_map(64)
    atmos = {"local": local_atmos(amap, 0, 1), "fields": [(2, 1, 1, "MEVA", np.zeros(amap.n_atmos))]}
    with pytest.raises(TypeError):
        Engine(c32.lf, 1, c32.methods, atmos=atmos)
    rm = {"n_dst": 4, "src": np.arange(64, dtype=np.int32), "dst": np.arange(64, dtype=np.int32) % 4,
          "w": np.ones(64), "fields": [(2, 1, 1, "MEVA", np.zeros(4))]}
    with pytest.raises(TypeError):
        Engine(c32.lf, 1, c32.methods, remaps=[rm])


def test_mixed_precision_bindings_rejected():
    case = build_case("CCLM", n=64, T=1)
    case.lf.dtype = "float32"  # float64 arrays in a float32 LocalFields
    with pytest.raises(TypeError):
        Engine(case.lf, 1, case.methods)


def test_set_precision_validates():
    lib = _lib.load()
    h = ctypes.c_void_p()
    gs = (ctypes.c_int32 * 3)(10, 10, 10)
    _lib.check(lib.fcx_create(0, 1, gs, ctypes.byref(h)))
    assert lib.fcx_set_precision(h, 2) == 1
    assert lib.fcx_set_precision(h, _lib.FCX_PRECISION_F32) == 0
    lib.fcx_destroy(h)


def test_remap_and_staging_options_before_commit():
    """FCX_OPT_REMAP_PACK (13: 0 never, 1 always, 2 auto), FCX_OPT_HOST_STAGING (15) and
    FCX_OPT_HOST_THREADS (16: 0..64) are validated without a GPU; the options retired in
    version 3 (6 page-locking of caller memory, 12/14 the in-launch carry hand-off) are
    accepted and ignored, and their query functions answer 0, so hosts that used them still
    run; an unknown option is rejected; fcx_remap_info is only answered after fcx_commit."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    gs = (ctypes.c_int32 * 3)(16, 16, 16)
    _lib.check(lib.fcx_create(0, 1, gs, ctypes.byref(h)))
    for v in (0, 1, 2):
        _lib.check(lib.fcx_set_option(h, 13, v))
    assert lib.fcx_set_option(h, 13, 3) == 1  # FCX_E_ARG
    for v in (0, 1):
        _lib.check(lib.fcx_set_option(h, 15, v))
    for v in (0, 1, 8, 64):
        _lib.check(lib.fcx_set_option(h, 16, v))
    assert lib.fcx_set_option(h, 16, 65) == 1
    assert lib.fcx_set_option(h, 16, -1) == 1
    for gone in (6, 12, 14):
        _lib.check(lib.fcx_set_option(h, gone, 1))
        _lib.check(lib.fcx_set_option(h, gone, 0))
    for v in (0, 1):
        _lib.check(lib.fcx_set_option(h, 19, v))  # FCX_OPT_LIB_SPANS
    assert lib.fcx_set_option(h, 19, 2) == 1
    assert lib.fcx_set_option(h, 20, 1) == 1  # FCX_E_ARG: unknown
    for v in (0, 1):
        _lib.check(lib.fcx_set_option(h, 18, v))  # FCX_OPT_DEFERRED_SCATTER
    b = ctypes.c_int64(7)
    _lib.check(lib.fcx_pinned_bytes(h, ctypes.byref(b)))
    assert b.value == 0
    b.value = 7
    _lib.check(lib.fcx_handoff_recoveries(h, ctypes.byref(b)))
    assert b.value == 0
    src = np.arange(16, dtype=np.int32)
    dst = src % 4
    w = np.ones(16)
    rid = ctypes.c_int32()
    _lib.check(lib.fcx_add_remap(h, 4, 16, src.ctypes.data, dst.ctypes.data, w.ctypes.data, ctypes.byref(rid)))
    sc, pk = ctypes.c_double(), ctypes.c_int32()
    assert lib.fcx_remap_info(h, rid.value, ctypes.byref(sc), ctypes.byref(pk)) == 2  # FCX_E_STATE
    assert lib.fcx_add_remap(h, 4, 1, src.ctypes.data, (dst + 4).ctypes.data, w.ctypes.data,
                             ctypes.byref(rid)) == 1  # a link outside the target grid
    lib.fcx_destroy(h)


def test_mock_rccl_stand_in_exports_the_entry_points_libfcx_binds():
    """The test-only librccl stand-in (tests/cpp/mock_rccl.cpp, FCX_RCCL_LIBRARY) that runs
    libfcx's N > 1 exchange with several ranks on one GPU: built by build(), and it exports
    every nccl* entry point libfcx resolves (fcx_engine.hip, rccl())."""
    path = os.path.join(ROOT, "components.flux_calculator_amd", "lib", "test", "libmock_rccl.so")
    assert os.path.exists(path), "make -C components.flux_calculator_amd mock-rccl"
    lib = ctypes.CDLL(path)
    for s in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclAllReduce", "ncclGetErrorString"):
        assert hasattr(lib, s), s
    uid = (ctypes.c_char * 128)()
    assert lib.ncclGetUniqueId(uid) == 0 and bytes(uid).startswith(b"/fcxmock-")


def test_one_cell_shared_on_both_sides_takes_one_slot():
    """A rank whose only atmosphere cell is shared with both neighbours uses the one slot of
    the cell (left == right, fcx.parallel.boundary_slots); two different slots are rejected
    with a named error before any collective."""
    case = build_case("CCLM", n=3, T=1)
    lib = _lib.load()
    idx = np.zeros(3, np.int32)
    w = np.full(3, 1.0 / 3)
    for left, right, ok in ((0, 0, True), (0, 1, False), (1, -1, True)):
        h = ctypes.c_void_p()
        gs = (ctypes.c_int32 * 3)(*case.lf.grid_size)
        _lib.check(lib.fcx_create(0, 1, gs, ctypes.byref(h)))
        try:
            _lib.check(lib.fcx_set_atmos_map(h, 1, ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(w.ctypes.data)))
            rc = lib.fcx_set_atmos_shared(h, ctypes.c_void_p(16), 2, 6, left, right)
            assert (rc == 0) == ok, (left, right, rc)
            if not ok:
                assert b"one boundary slot" in lib.fcx_last_error()
        finally:
            lib.fcx_destroy(h)


def test_abort_handler_receives_the_message():
    """fcx_set_abort_handler / fcx_abort (the oasis_abort hook of the drop-in,
    flux_calculator.F90:883-887): without a handler fcx_abort reports FCX_E_STATE; a
    registered one gets the message; NULL unregisters.  Host-side only."""
    lib = _lib.load()
    got = []
    proto = ctypes.CFUNCTYPE(None, ctypes.c_char_p)
    cb = proto(lambda msg: got.append(msg.decode()))
    assert lib.fcx_set_abort_handler(None) == 0
    assert lib.fcx_abort(b"nobody listens") == 2
    assert lib.fcx_set_abort_handler(ctypes.cast(cb, ctypes.c_void_p)) == 0
    try:
        assert lib.fcx_abort(b"flux engine error in fcx_step: boom") == 0
    finally:
        assert lib.fcx_set_abort_handler(None) == 0
    assert got == ["flux engine error in fcx_step: boom"]
    assert lib.fcx_abort(b"again") == 2 and len(got) == 1


def test_group_and_comm_queries_validate_arguments():
    """fcx_last_group_size / fcx_comm_verify reject NULL handles with FCX_E_ARG (no GPU
    needed); the round-5 overlapped exchange (fcx_run_group_exchange) is gone from the ABI."""
    lib = _lib.load()
    m = ctypes.c_int32()
    assert lib.fcx_last_group_size(None, ctypes.byref(m)) == 1
    assert lib.fcx_comm_verify(None, 1) == 1
    assert not hasattr(lib, "fcx_run_group_exchange") and not hasattr(lib, "fcx_comm_overlapped")
    assert lib.fcx_step_async(None, 3, 0) != 0
