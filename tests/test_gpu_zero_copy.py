"""Host memory transports, each hazard forced deterministically.

Until round 2 the engine reached caller heap memory through hipHostRegister: kernels used
registered arrays in place, later only DMAs did, and a process-wide registry shared one
registration between engines that asked for the same virtual byte range.  Three wrong
results came out of that (round 1: MEVA stores that never reached the host array; round 2:
an HLAT computed from MEVA one 4 KiB page off; an illegal memory access in a DMA out of
fresh heap arrays).  A registration pins the physical pages behind a range at the moment it
is made, while everything that looks it up -- the registry, the runtime's own map of host
memory -- goes by virtual address; once the allocation behind the range is freed and its
address handed out again (glibc reuses a freed mapping of the same size at the same
address), a lookup by address finds a registration of pages that no longer back it.  Since
round 3 nothing of the caller's memory is registered or mapped: heap arrays move through the
engine's own page-locked staging arena, read and written by host copies at the arrays'
virtual addresses at every step.  Set up here on purpose:

  * the virtual address of live engines' arrays unmapped and mapped again with new contents
    (MAP_FIXED) before a second engine binds the same addresses;
  * an output whose page meets another live engine's arrays, before and after that engine
    is closed;
  * an engine dropped without close() and collected by the garbage collector between the
    commit and the step of a new engine over fresh arrays;
  * two live engines over the same arrays, one closed before the other steps;
  * library arrays (fcx_host_malloc) in place with non-temporal and plain accesses, over
    several steps with the host rewriting inputs, and a per-call chain where each kernel
    reads the previous kernel's outputs in host memory;
  * caller heap arrays are never used in place, whatever FCX_OPT_ZERO_COPY says.
"""
import gc

import numpy as np
import pytest

import oracle_lib
from parity import assert_parity

pytestmark = pytest.mark.gpu

fcx = pytest.importorskip("fcx")
from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.local_field import rehome  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402
from fcx import host_alloc  # noqa: E402

T_STEP = 3600
PAGE = 4096


def engine_for(case, **opts):
    return Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                  averages=case.averages, options=opts)


def reset_outputs(case):
    for k in case.outputs:
        case.lf.field[k][:] = np.nan


def check(case, label):
    ref = oracle_lib.run_case(case, "c", current_step_time=T_STEP)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    assert_parity(got, ref, label=label)


def carve(cases, first_key=None):
    """Re-home the arrays of several cases back to back in ONE heap buffer, each case's
    arrays contiguous, consecutive cases meeting inside one page (8-B apart), so that the
    last array of case k and the first array of case k+1 share a page.  first_key puts that
    (s, g, name) array first in every case."""
    sizes = []
    for c in cases:
        seen = {}
        for a in c.lf.field.values():
            seen[id(a)] = a.nbytes
        sizes.append(sum(seen.values()))
    total = sum(sizes) + 8 * len(cases) + 2 * PAGE
    buf = np.empty(total // 8 + 1, dtype=np.float64)
    off = (-buf.ctypes.data) % PAGE + 8 * 17  # start mid-page
    for c, sz in zip(cases, sizes):
        rehome(c.lf, buf, off, first_key=first_key)
        off += sz + 8
    return buf


def test_output_page_shared_with_another_live_engine():
    """Case B's MEVA begins on the page where case A's arrays end, both engines live."""
    a = build_case("MOM5", n=4097, T=1)
    b = build_case("MOM5", n=4097, T=1)
    keep = carve([a, b], first_key=(1, 1, "MEVA"))
    ea = engine_for(a)
    eb = engine_for(b)
    eb.step(PHASE_ALL, T_STEP)
    check(b, "B with A live")
    ea.step(PHASE_ALL, T_STEP)
    check(a, "A")
    ea.close()
    reset_outputs(b)
    eb.step(PHASE_ALL, T_STEP)
    check(b, "B after A closed")
    eb.close()
    del keep


class _Cycle:
    def __init__(self, eng, case):
        self.eng, self.case, self.me = eng, case, self


def test_engine_collected_between_commit_and_step():
    """An engine only the cyclic garbage collector frees (never closed) is destroyed after a
    new engine over fresh arrays has committed and before it steps."""
    for n in (4097, 10_007):
        a = build_case("MOM5", n=n, T=1)
        _Cycle(engine_for(a), a)  # unreachable, alive until gc.collect()
        del a
        b = build_case("MOM5", n=n, T=1)
        eb = engine_for(b)
        gc.collect()  # the old engine's fcx_destroy runs here
        eb.step(PHASE_ALL, T_STEP)
        check(b, f"n={n} after collecting the old engine")
        eb.close()


def test_two_engines_over_the_same_arrays():
    """Two live engines over the same arrays; closing the first leaves the second intact."""
    c = build_case("CCLM", n=4097, T=1, bias=True)
    e1 = engine_for(c)
    e2 = engine_for(c)
    e1.step(PHASE_ALL, T_STEP)
    check(c, "first engine")
    e1.close()
    reset_outputs(c)
    e2.step(PHASE_ALL, T_STEP)
    check(c, "second engine after the first closed")
    e2.close()


@pytest.mark.parametrize("nontemporal", [0, 1])
def test_host_mapped_stores(nontemporal):
    """Library arrays in place: the engine drops the non-temporal hint for mapped fields
    whatever FCX_OPT_NONTEMPORAL says; the results are the same either way."""
    for v in ("CCLM", "MOM5", "RCO"):
        c = build_case(v, n=4097, T=1)
        with host_alloc.Arena() as arena:
            arena.adopt(c.lf)
            e = engine_for(c, zero_copy=1, nontemporal=nontemporal)
            assert e.zero_copy_active()
            for _ in range(3):
                reset_outputs(c)
                e.step(PHASE_ALL, T_STEP)
                check(c, f"{v} nt={nontemporal}")
            e.close()


def test_library_arrays_per_call_chain():
    """The per-call reference subroutines on library arrays in place: each kernel reads what
    the previous call's kernel wrote to host memory (QSUR -> MEVA -> HLAT -> averages)."""
    from fcx.basic import IDX

    STEP = 3600 * 24 * 40
    case = build_case("CCLM", n=5_003, T=2, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP)
    with host_alloc.Arena() as arena:
        arena.adopt(case.lf)
        reset_outputs(case)
        eng = Engine(case.lf, 2, case.methods, corrections=case.corrections, averages=case.averages,
                     options={"zero_copy": 1})
        assert eng.zero_copy_active()
        lib, h = eng.lib, eng.h
        assert lib.fcx_calc_flux_radiation_blackbody(h) == 0
        for g in (1, 2, 3):
            assert lib.fcx_calc_spec_vapor_surface(h, g) == 0
        assert lib.fcx_calc_flux_mass_evap(h, STEP) == 0
        assert lib.fcx_calc_flux_heat_latent(h) == 0
        assert lib.fcx_calc_flux_heat_sensible(h) == 0
        assert lib.fcx_calc_flux_momentum_east(h, 2) == 0
        assert lib.fcx_calc_flux_momentum_north(h, 3) == 0
        for ph, g, name in case.averages:
            assert lib.fcx_average_across_surface_types(h, g, IDX[name]) == 0
        got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
        eng.close()
    assert_parity(got, ref, label="library arrays per call")


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("n", [4097, 32_768])
@pytest.mark.parametrize("transport", ["spans", "zero_copy"])
def test_library_pinned_arrays(variant, n, transport):
    """Arrays allocated by fcx_host_malloc (page-locked and mapped by the library itself, no
    registration of caller memory): used in place by default at these sizes (auto zero-copy);
    with FCX_OPT_ZERO_COPY 0 the span transport moves them (device mirrors laid out like the
    host memory, one copy per run of adjacent arrays)."""
    c = build_case(variant, n=n, T=2, bias=True)
    with host_alloc.Arena() as arena:
        arena.adopt(c.lf)
        e = engine_for(c, zero_copy=0) if transport == "spans" else engine_for(c)
        assert e.zero_copy_active() == (transport == "zero_copy")
        if transport == "spans":
            up, down = e.span_runs()
            assert 1 <= up <= 4 and down == 1, (up, down)  # (unread inputs between read ones: gaps)
        assert e.staging_bytes() == 0  # library memory: no staging arena either
        for k in range(3):
            reset_outputs(c)
            e.step(PHASE_ALL, T_STEP)
            check(c, f"{variant} step {k}")
            for key in ("TSUR", "PSUR"):  # fresh inputs between steps reach the kernel
                arr = c.lf.field[(1, 1, key)]
                arr[:] = arr * (1.0 + 1e-4)
        e.close()


@pytest.mark.parametrize("zero_copy", [0, 1, 2])
@pytest.mark.parametrize("staging", [0, 1])
def test_heap_arrays_never_used_in_place(zero_copy, staging):
    """Caller heap arrays are never what a kernel addresses, whatever FCX_OPT_ZERO_COPY says:
    with zero-copy and the staging arena the kernels use the library's mapped arena image of
    them in place (the small-grid default), otherwise device mirrors."""
    c = build_case("CCLM", n=4097, T=1)
    e = engine_for(c, zero_copy=zero_copy, host_staging=staging)
    assert e.zero_copy_active() == bool(zero_copy and staging)
    for (s, g, name), a in c.lf.field.items():
        assert e.device_ptr(s, g, name) != a.ctypes.data, (s, g, name)
    for k in range(3):
        reset_outputs(c)
        e.step(PHASE_ALL, T_STEP)
        check(c, f"step {k}")
    e.close()


def _libc():
    import ctypes

    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return libc


PROT_RW, MAP_PRIVATE_ANON, MAP_FIXED = 0x3, 0x22, 0x10


@pytest.mark.parametrize("variant", ["CCLM", "MOM5"])
def test_recycled_virtual_address_between_engines(variant):
    """Engine A binds arrays in an anonymous mapping; the mapping is then replaced at the same
    virtual address (MAP_FIXED: new zero pages) and filled with another case's inputs while A
    is alive; engine B binds the same addresses.  Both engines must compute from the new
    contents -- the address-keyed registration sharing of round 2 would have handed B (and A)
    the pages of the old mapping."""
    import ctypes

    libc = _libc()
    a = build_case(variant, n=10_007, T=1, bias=True, seed=3)
    b = build_case(variant, n=10_007, T=1, bias=True, seed=4)
    b.corrections = a.corrections  # engine state (copied at set-up), not memory at the addresses
    size = 2 * 1024 * 1024
    addr = libc.mmap(None, size, PROT_RW, MAP_PRIVATE_ANON, -1, 0)
    assert addr not in (None, ctypes.c_void_p(-1).value)
    view = np.frombuffer((ctypes.c_char * size).from_address(addr), dtype=np.uint8)
    try:
        end_a = rehome(a.lf, view, 8 * 3)  # mid-page start
        ea = engine_for(a)
        ea.step(PHASE_ALL, T_STEP)
        check(a, "A before the remap")
        # the same virtual range, new physical pages, B's inputs at A's addresses
        again = libc.mmap(addr, size, PROT_RW, MAP_PRIVATE_ANON | MAP_FIXED, -1, 0)
        assert again == addr
        assert rehome(b.lf, view, 8 * 3) == end_a
        for key in a.lf.field:  # one layout: A's arrays are B's arrays now
            assert a.lf.field[key].ctypes.data == b.lf.field[key].ctypes.data
        eb = engine_for(b)
        eb.step(PHASE_ALL, T_STEP)
        check(b, "B at the recycled addresses")
        reset_outputs(b)
        ea.step(PHASE_ALL, T_STEP)  # A reads the new contents too
        check(b, "A after the remap")
        ea.close()
        reset_outputs(b)
        eb.step(PHASE_ALL, T_STEP)
        check(b, "B after A closed")
        eb.close()
    finally:
        libc.munmap(addr, size)


SPAN_MODES = ["step", "step_async", "per_call", "upload_field"]


def _run_mode(case, eng, mode, t):
    lib, h = eng.lib, eng.h
    if mode == "step":
        eng.step(PHASE_ALL, t)
    elif mode == "step_async":
        eng.step_async(PHASE_ALL, t)
        eng.synchronize()
    elif mode == "upload_field":
        outs = {id(case.lf.field[k]) for k in case.outputs}
        seen = set()
        for key, a in case.lf.field.items():
            if id(a) not in outs and id(a) not in seen and key[0] >= 1:
                seen.add(id(a))
                eng.upload_field(*key)
        eng.step(PHASE_ALL, t)
    else:
        from fcx.basic import IDX

        assert lib.fcx_calc_flux_radiation_blackbody(h) == 0, lib.fcx_last_error()
        for g in (1, 2, 3):
            assert lib.fcx_calc_spec_vapor_surface(h, g) == 0
        assert lib.fcx_calc_flux_mass_evap(h, t) == 0
        assert lib.fcx_calc_flux_heat_latent(h) == 0
        assert lib.fcx_calc_flux_heat_sensible(h) == 0
        assert lib.fcx_calc_flux_momentum_east(h, 2) == 0
        assert lib.fcx_calc_flux_momentum_north(h, 3) == 0
        for ph, g, name in case.averages:
            assert lib.fcx_average_across_surface_types(h, g, IDX[name]) == 0


@pytest.mark.parametrize("mode", SPAN_MODES)
@pytest.mark.parametrize("variant,T,n", [("CCLM", 1, 32_768), ("MOM5", 2, 4_099), ("RCO", 3, 1_001),
                                         ("CCLM", 2, 600_000)])
def test_span_transport_bit_identical_to_heap_arrays(variant, T, n, mode):
    """the span transport of fcx_host_malloc arrays (one upload and one
    download per run of adjacent arrays; the chunk pipeline at 600,000 cells) gives outputs
    bit-identical to the same case from caller heap arrays, in every way a host drives the
    engine: fcx_step, fcx_step_async + fcx_synchronize, the per-call subroutines, fields
    handed over one by one -- over two steps with the inputs changed in between."""
    t = 3600 * 24 * 31
    heap = build_case(variant, n=n, T=T, bias=True, seed=17)
    lib_case = build_case(variant, n=n, T=T, bias=True, seed=17)
    with host_alloc.Arena() as arena:
        arena.adopt(lib_case.lf)
        e_heap = engine_for(heap)
        e_lib = engine_for(lib_case, zero_copy=0)  # (the span transport; auto would use them in place)
        assert not e_lib.zero_copy_active() and e_lib.staging_bytes() == 0
        for step in range(2):
            for c in (heap, lib_case):
                reset_outputs(c)
                if step:
                    for key in ("TSUR", "TATM", "UATM"):
                        for s in range(0, T + 1):
                            if (s, 1, key) in c.lf.field:
                                a = c.lf.field[(s, 1, key)]
                                a[:] = a * (1.0 + 1e-4)
            _run_mode(heap, e_heap, mode, t)
            _run_mode(lib_case, e_lib, mode, t)
            for k in heap.outputs:
                a, b = np.asarray(heap.lf.field[k]), np.asarray(lib_case.lf.field[k])
                assert np.array_equal(a, b, equal_nan=True), (k, mode, step)
        ref = oracle_lib.run_case(lib_case, "c", current_step_time=t)
        got = {k: np.array(lib_case.lf.field[k], copy=True) for k in lib_case.outputs}
        assert_parity(got, ref, label=f"spans {variant} T={T} {mode}")
        e_heap.close()
        e_lib.close()


def test_span_runs_follow_the_allocation_order():
    """Arrays allocated inputs first, then outputs (the reference's order: allocate_localvar
    for every input, flux_calculator.F90:436-560, then do_prepare_calculation for the outputs,
    prepare:36-42) move as ONE upload and ONE download per step; the same arrays allocated
    with the outputs interleaved between the inputs take more copies, and unbound gaps between
    outputs are never written by a download."""
    c = build_case("CCLM", n=32_768, T=1, bias=False, seed=3)
    with host_alloc.Arena() as arena:
        arena.adopt(c.lf)  # dict order: inputs, then outputs
        e = engine_for(c, zero_copy=0)
        assert e.span_runs() == (1, 1)
        e.close()
    c2 = build_case("CCLM", n=32_768, T=1, bias=False, seed=3)
    outs = {id(c2.lf.field[k]) for k in c2.outputs}  # (this case's own arrays: ids of c's may be reused)
    with host_alloc.Arena() as arena:
        moved, guards = {}, []
        for key, a in list(c2.lf.field.items()):  # interleaved: a guard block after every output
            if id(a) in moved:
                c2.lf.field[key] = moved[id(a)]
                continue
            v = arena.empty(a.shape[0], a.dtype)
            v[:] = a
            moved[id(a)] = v
            c2.lf.field[key] = v
            if id(a) in outs:
                g = arena.empty(64)
                g[:] = 12345.0
                guards.append(g)
        e = engine_for(c2, zero_copy=0)
        up, down = e.span_runs()
        assert len(guards) == len(outs) and down > 1, (len(guards), up, down)
        reset_outputs(c2)
        e.step(PHASE_ALL, T_STEP)
        check(c2, "spans with guards between the outputs")
        for g in guards:
            assert np.all(g == 12345.0)
        e.close()


def test_host_malloc_blocks_follow_the_call_order():
    """fcx_host_malloc carves 256-B aligned blocks from page-locked slabs in call order (what
    lets the span transport move adjacent arrays as one copy): consecutive blocks are
    adjacent, freeing the last block lets the next call take its place, a freed block in the
    middle is not handed out again while its slab lives, a block that does not fit opens a new
    slab, and fcx_host_free names a pointer it does not own."""
    import ctypes

    from fcx import _lib

    lib = _lib.load()
    MB = 1 << 20

    def malloc(n):
        p = ctypes.c_void_p()
        _lib.check(lib.fcx_host_malloc(n, ctypes.byref(p)))
        assert p.value and p.value % 256 == 0
        ctypes.memset(p.value, 0x5A, max(n, 1))  # page-locked host memory the caller may write
        return p.value

    def free(p):
        _lib.check(lib.fcx_host_free(ctypes.c_void_p(p)))

    big = malloc(33 * MB)  # fits no partly used 32-MB slab: a fresh 34-MB slab, current from now on
    p1 = malloc(1000)
    p2 = malloc(5000)
    assert p1 == big + 33 * MB and p2 == p1 + 1024
    free(p2)
    p3 = malloc(100)
    assert p3 == p2  # the tail block's place is reused
    free(p1)
    p4 = malloc(100)
    assert p4 == p3 + 256  # the hole p1 left is not
    p5 = malloc(2 * MB)  # ~1 MB left in the slab: a new one
    assert not (big <= p5 < big + 34 * MB)
    for p in (big, p3, p4, p5):
        free(p)
    free(None)  # NULL is a no-op, as free(3)
    foreign = ctypes.create_string_buffer(64)
    assert lib.fcx_host_free(ctypes.cast(foreign, ctypes.c_void_p)) != 0
    assert b"fcx_host_malloc" in lib.fcx_last_error()
