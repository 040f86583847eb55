/*
 * fcx.h -- C ABI of the MI355X exchange-grid flux engine (libfcx.so).
 *
 * This is the drop-in boundary for the per-coupling-step flux path of the IOW-ESM
 * flux_calculator.  It replaces the compute of module flux_calculator_calculate
 * (/root/reference/src/flux_calculator_calculate.F90) and do_regridding
 * (flux_calculator_basic.F90:463-522); the Fortran host keeps its data model, OASIS
 * put/get and namcouple surface.  The iso_c_binding shim that binds these entry points
 * under the reference subroutine names is
 * components.flux_calculator_amd/fortran/flux_calculator_calculate.F90.
 *
 * Plain C: integers, doubles and opaque handles only.  Every entry point returns an int
 * status (FCX_OK == 0); on failure fcx_last_error() returns a message (thread-local).
 * The reference calc_* never fail at run time (validation happens in
 * flux_calculator_prepare.F90); here validation happens in fcx_commit and later calls
 * only fail on HIP errors or misuse.  Not re-entrant per engine (one engine per rank and
 * GPU, calls serialised by the host loop, as in the reference).
 */
#ifndef FCX_H
#define FCX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FCX_VERSION 1
#define FCX_MAX_SURFACE_TYPES 10 /* flux_calculator_basic.F90:28 */
#define FCX_NUM_VARS 35          /* flux_calculator_basic.F90:42 */

/* Variable ids: identical to the reference idx_* values (flux_calculator_basic.F90:526-568). */
enum fcx_var {
  FCX_ALBE = 1, FCX_ALBA, FCX_AMOI, FCX_AMOM, FCX_FARE, FCX_FICE, FCX_PATM, FCX_PSUR,
  FCX_QATM, FCX_TATM, FCX_TSUR, FCX_UATM, FCX_VATM, FCX_U10M, FCX_V10M,
  FCX_CMOM, FCX_CMOI, FCX_CHEA, FCX_QSUR, FCX_HLAT, FCX_HSEN,
  FCX_MEVA, FCX_MPRE, FCX_MRAI, FCX_MSNO,
  FCX_RBBR, FCX_RLWD, FCX_RLWU, FCX_RSID, FCX_RSIU, FCX_RSIN, FCX_RSDD, FCX_RSDR,
  FCX_UMOM, FCX_VMOM
};

/* which_grid: 1 = t_grid, 2 = u_grid, 3 = v_grid (flux_calculator_basic.F90:64) */
enum fcx_grid { FCX_T_GRID = 1, FCX_U_GRID = 2, FCX_V_GRID = 3 };

/* Method strings of the namelist which_* tables (flux_calculator.F90:99-107). */
enum fcx_method {
  FCX_NONE = 0, FCX_ZERO, FCX_COPY, FCX_CCLM, FCX_MOM5, FCX_RCO, FCX_WATER, FCX_ICE, FCX_STBO
};

/* The which_* tables, in the order of the namelist (flux_calculator.F90:99-107). */
enum fcx_flux {
  FCX_SPEC_VAPOR_SURFACE_T = 0, FCX_SPEC_VAPOR_SURFACE_U, FCX_SPEC_VAPOR_SURFACE_V,
  FCX_FLUX_MASS_EVAP, FCX_FLUX_HEAT_LATENT, FCX_FLUX_HEAT_SENSIBLE, FCX_FLUX_MOMENTUM,
  FCX_FLUX_RADIATION_BLACKBODY, FCX_NUM_FLUXES
};

/* Coupling-step phases (flux_calculator.F90:872-936 early, :942-1026 normal). */
enum fcx_phase { FCX_PHASE_EARLY = 1, FCX_PHASE_NORMAL = 2, FCX_PHASE_ALL = 3 };

/* Regridding matrices (flux_calculator.F90:330-337). */
enum fcx_regrid { FCX_U_TO_T = 0, FCX_V_TO_T, FCX_T_TO_U, FCX_T_TO_V };

enum fcx_status {
  FCX_OK = 0, FCX_E_ARG = 1, FCX_E_STATE = 2, FCX_E_UNSUPPORTED = 3, FCX_E_HIP = 4,
  FCX_E_MISSING = 5, FCX_E_NOMEM = 6
};

/* fcx_bind_field flags */
#define FCX_MEM_HOST   0x0 /* ptr is a host array owned by the caller (Fortran)       */
#define FCX_MEM_DEVICE 0x1 /* ptr is device memory owned by the caller (zero copy)     */
#define FCX_ALLOCATED  0x2 /* realarray%allocated (basic:88): an own array, not alias */

/* fcx_set_corrections layouts */
#define FCX_CORR_CELL_MAJOR  0 /* Fortran corrections(1,12,grid_size(1)) (bias:29-30,191) */
#define FCX_CORR_MONTH_MAJOR 1 /* [12][grid_size(1)] (the device layout)                 */

typedef struct fcx_engine fcx_engine;

const char *fcx_last_error(void);
int fcx_version(void);

/* The host's abort routine for errors that must end the coupled run, not just this rank:
 * the reference turns them into oasis_abort(comp_id, comp_name, msg)
 * (flux_calculator.F90:883-887, 930-934, 960-964).  The Fortran drop-in module calls
 * fcx_abort(message) on a failed call or a contract violation before its own ERROR STOP, so
 * a host that registers a routine calling oasis_abort (or MPI_Abort) takes the other
 * components down with it instead of leaving them waiting in their next exchange.
 * Process-wide; NULL unregisters.  fcx_abort returns FCX_E_STATE when none is registered,
 * FCX_OK when the handler returned. */
typedef void (*fcx_abort_handler)(const char *message);
int fcx_set_abort_handler(fcx_abort_handler handler);
int fcx_abort(const char *message);

/* trim(method)=='CCLM' etc. on a blank-padded Fortran CHARACTER(len=20); -1 if unknown */
int fcx_method_from_string(const char *s, size_t len);

/* datetime_helpers.get_current_date (pyfort/datetime_helpers.py:4-13): calendar month of
 * init_date (YYYYMMDD) + seconds.  Replaces the Fortran->C->CPython round trip of
 * calc:66-73. */
int fcx_current_month(int32_t init_date, int64_t seconds, int32_t *month);

/* ---- engine set-up (after flux_calculator.F90:761, when allocations are final) ---- */
int fcx_create(int device, int num_surface_types, const int32_t grid_size[3], fcx_engine **out);
int fcx_destroy(fcx_engine *e);
/* hipStream_t to run on (default: a stream owned by the engine) */
int fcx_set_stream(fcx_engine *e, void *hip_stream);
/* methods(my_bottom_model, surface_type) of one which_* table */
int fcx_set_method(fcx_engine *e, int flux, int surface_type, int method);
/* local_field(surface_type, grid)%var(var)%field => ptr(1:n).  Identical pointers in
 * several slots are aliases (basic:334-358, prepare:36-38) and share one device buffer. */
int fcx_bind_field(fcx_engine *e, int surface_type, int grid, int var, double *ptr, int64_t n,
                   int flags);
/* bias_corrections: lcorrections(E_MASS_EVAP_CORRECTION), init_date, corrections(1,:,:) */
int fcx_set_corrections(fcx_engine *e, int enabled, int32_t init_date, const double *corr,
                        int64_t n, int layout);
/* sparse_regridding_matrix (basic:117-122): 1-based, rank-local, offset-corrected links */
int fcx_set_regrid_matrix(fcx_engine *e, int which, int64_t num_elements, const int32_t *src_index,
                          const int32_t *dst_index, const double *weight);
/* realarray%put_to_{t,u,v}_grid of (surface_type, grid, var): bit0 t, bit1 u, bit2 v */
int fcx_set_put_to(fcx_engine *e, int surface_type, int grid, int var, int mask);
/* register a type-0 output that is averaged before its oasis_put (flux_calculator.F90:
 * 911-918 early, 1001-1008 normal).  Follows the P7 trigger: only applied when the type-0
 * array is FCX_ALLOCATED and surface type 2 exists. */
int fcx_add_average(fcx_engine *e, int phase, int grid, int var);
/* arithmetic/storage type of the engine's fields.  FCX_PRECISION_F64 (default) is the
 * reference's -r8 build (build_hlrnb.sh:26).  FCX_PRECISION_F32: every pointer given to
 * fcx_bind_field / fcx_add_atmos_field / returned by fcx_device_ptr addresses float arrays
 * (the double* parameter type then only carries the address) and the kernels compute in
 * fp32 -- the SURVEY.md 8d config-5 variant, half the HBM bytes per cell.  Corrections are
 * still passed as double and rounded once at commit.  do_regridding runs in fp32 with the
 * matrix weights rounded once (the single-precision build's REAL(wp) arithmetic,
 * basic:117-122, 463-522).  The atmosphere accumulation and the remaps read the fp32 fields
 * and write fp32 outputs (fcx_add_atmos_field / fcx_add_remap_field then take float arrays)
 * but weigh and sum in fp64, as OASIS maps in double; the shared boundary buffer of
 * fcx_set_atmos_shared stays double.  Call before fcx_commit. */
enum fcx_precision { FCX_PRECISION_F64 = 0, FCX_PRECISION_F32 = 1 };
int fcx_set_precision(fcx_engine *e, int precision);
/* validate (flux_calculator_prepare.F90 rules), allocate device mirrors, build plans */
int fcx_commit(fcx_engine *e);
/* before fcx_commit, host only (no GPU): validate, then build every launch plan the engine can
 * take -- the whole phases, the per-call subroutines, the regridding sequence, the explicit
 * averages -- and audit each against the kernels' load predicates: a computed flux whose input
 * the planner did not bind is a named FCX_E_STATE error (the same audit runs on every plan
 * fcx_commit and the later calls build, before its first launch) */
int fcx_plan_check(fcx_engine *e);

/* ---- per coupling step: fused path ---- */
int fcx_upload(fcx_engine *e, int phase);   /* H2D of host-bound inputs of the phase  */
int fcx_run(fcx_engine *e, int phase, int32_t current_step_time); /* device compute  */
int fcx_download(fcx_engine *e, int phase); /* D2H of host-bound outputs of the phase */
/* fcx_run of several engines on one device (e.g. one per bottom-model variant), in the order
 * given: the flux passes of those whose phase is one fused T = 1 launch of the same shape on
 * the same stream go out as ONE launch (at most 4 engines; the others run as fcx_run), so a
 * step pays the launch ramp and drain once.  Results are those of fcx_run of each, bit for
 * bit. */
int fcx_run_group(fcx_engine *const *engines, int n_engines, int phase, int32_t current_step_time);
/* engines in the merged launch of the engine's last fcx_run_group (0: it ran as fcx_run).
 * Every engine's work after its launch (fix-up, accumulation, the boundary exchange of an
 * attached communicator, remaps) runs in LIST order whichever engines were merged, so the
 * per-engine collectives of fcx_set_comm keep the same order on every rank. */
int fcx_last_group_size(fcx_engine *e, int32_t *members);
/* the three above; with host-bound fields pipelined over cell chunks (FCX_OPT_PIPELINE_CHUNKS) */
int fcx_step(fcx_engine *e, int phase, int32_t current_step_time);
/* waits for the engine's stream; the caller's host arrays hold the downloaded outputs once it
 * returns.  fcx_download fills caller heap arrays itself (it waits for the stream); with
 * FCX_OPT_DEFERRED_SCATTER they are filled from the staging arena here.  fcx_step and the
 * per-call subroutines end with it. */
int fcx_synchronize(fcx_engine *e);
/* fcx_step without its final wait (the asynchronous phase): when it returns the engine holds
 * the inputs (caller heap arrays are copied into the staging arena inside the call, so the
 * host may overwrite them), the launch and the output DMAs are queued, and the caller's
 * output arrays are filled by the next fcx_synchronize.  Inputs in fcx_host_malloc memory
 * are read in place until then.  A host starts several engines this way from one thread (each
 * on its own stream), or overlaps its own work -- another component's exchange -- with the
 * step.  Host-bound grids of at least two pipeline chunks complete inside the call. */
int fcx_step_async(fcx_engine *e, int phase, int32_t current_step_time);
/* One input field handed over as the host receives it (oasis_get of field j, then
 * fcx_upload_field): its host array is copied into the staging arena and DMAed to its
 * mirror by the engine's upload thread while the host goes on to receive the next field
 * (flux_calculator.F90:872-897, 938-966: the reference gets the fields one by one).  The
 * upload thread copies the array at some point before the next engine call (any but
 * fcx_upload_field) returns, so the array must not change until that call returns; from
 * then on the host may overwrite it -- every call first waits for the handed-over fields.
 * fcx_upload / fcx_step / fcx_step_async then move only the phase's remaining inputs.
 * Aliases (one array in several slots) are handed over once.  If a hand-over fails, the
 * next call returns its error and no field counts as handed over, so a retried step moves
 * every input again. */
int fcx_upload_field(fcx_engine *e, int surface_type, int grid, int var);

/* ---- per call: the reference subroutines one by one (exact drop-in semantics; each
 * call uploads what it reads, computes, downloads what it writes, and synchronises) ---- */
int fcx_calc_spec_vapor_surface(fcx_engine *e, int which_grid);            /* calc:25  */
int fcx_calc_flux_mass_evap(fcx_engine *e, int32_t current_step_time);     /* calc:54  */
int fcx_calc_flux_heat_latent(fcx_engine *e);                              /* calc:124 */
int fcx_calc_flux_heat_sensible(fcx_engine *e);                            /* calc:156 */
int fcx_calc_flux_momentum_east(fcx_engine *e, int which_grid);            /* calc:212 */
int fcx_calc_flux_momentum_north(fcx_engine *e, int which_grid);           /* calc:265 */
int fcx_calc_flux_radiation_blackbody(fcx_engine *e);                      /* calc:320 */
int fcx_distribute_shortwave_radiation_flux(fcx_engine *e);                /* calc:347 */
int fcx_average_across_surface_types(fcx_engine *e, int which_grid, int var); /* calc:368 */
int fcx_do_regridding(fcx_engine *e, int var, int surface_type);           /* basic:463 */

/* ---- device-resident use and measurement ---- */
/* device buffer behind a slot (NULL if unbound).  Cell j of it sits at element
 * (j / tile) * tile_stride + j % tile (fcx_device_layout); tile_stride == tile means the
 * buffer is one contiguous array. */
int fcx_device_ptr(fcx_engine *e, int surface_type, int grid, int var, double **dptr);
/* layout of the engine-owned field mirrors (after fcx_commit): cells in tiles of `tile`
 * elements, consecutive tiles of one array `tile_stride` elements apart (FCX_OPT_TILED_LAYOUT) */
int fcx_device_layout(fcx_engine *e, int64_t *tile, int64_t *tile_stride);
/* device time (hipEvents on the engine stream) of the kernels of the last fcx_run;
   needs FCX_OPT_TIMING = 1 */
int fcx_last_kernel_ms(fcx_engine *e, float *ms);
/* bytes of the engine's page-locked staging arena for caller heap arrays (0: none): one host
 * image per device pool that holds a heap array's mirror, allocated at fcx_commit (the
 * pinned footprint: ~the mirrors' size, e.g. 2.2-2.6 GB per 10M-cell CCLM engine).  A pool
 * whose image cannot be page-locked takes the direct path instead and is not counted. */
int fcx_staging_bytes(fcx_engine *e, int64_t *bytes);
/* retired in version 3, kept for one release: always 0 (nothing of the caller's memory is
 * page-locked; the in-launch carry hand-off is gone) */
int fcx_pinned_bytes(fcx_engine *e, int64_t *bytes);
int fcx_handoff_recoveries(fcx_engine *e, int64_t *count);
/* bytes of host arrays the kernels use in place (FCX_OPT_ZERO_COPY) */
int fcx_zero_copy_bytes(fcx_engine *e, int64_t *bytes);
/* copies one fcx_step(phase) makes of the engine's fcx_host_malloc arrays with the span
 * transport (FCX_OPT_LIB_SPANS): uploads, downloads (0 / 0 when no array takes it) */
int fcx_span_runs(fcx_engine *e, int phase, int32_t *h2d_copies, int32_t *d2h_copies);
/* algorithmic HBM bytes of one fcx_run(phase) (each distinct array read once, written once) */
int fcx_algorithmic_bytes(fcx_engine *e, int phase, int64_t *bytes);

/* ---- exchange-grid -> atmosphere accumulation ----
 * What OASIS3-MCT does on oasis_put of the type-0 fields ('S A xxxx 00',
 * create_namcouple.F90:92-98): out[a] = sum_x weight[x] * field[x] over the local t-grid
 * exchange cells x of atmosphere cell a, summed in increasing x.  Ranks own contiguous
 * exchange ranges, so only the first and last local atmosphere cells can be shared with a
 * neighbour rank; their partial sums go to `shared` slots that ONE all-reduce (sum) over
 * all ranks completes, after which fcx_atmos_finish writes them back. */
/* atmos_index[x]: 0-based local atmosphere cell of exchange cell x (grid_size(1) entries) */
int fcx_set_atmos_map(fcx_engine *e, int64_t n_atmos, const int32_t *atmos_index,
                      const double *weight);
/* accumulate slot (surface_type, grid, var) into out[n_atmos] at the end of `phase` */
int fcx_add_atmos_field(fcx_engine *e, int phase, int surface_type, int grid, int var,
                        double *out, int flags);
/* shared: device buffer [n_boundaries][stride] (zero on entry, re-zeroed by finish); the
 * rank's first local atmosphere cell is boundary `left` (-1: not shared), its last one
 * boundary `right`; field f of the accumulation uses column f (f < stride).  Boundary m - 1
 * is the one just before rank m's cells: left = rank - 1, right = (next rank with cells) - 1
 * (a rank with an empty task, io:101-104, sits between two slots' owners without one).
 * Every rank that holds part of one atmosphere cell uses ONE slot for it, the slot of the
 * first rank boundary inside the cell: a rank whose cells all lie in one atmosphere cell
 * shared with both neighbours has left == right (fcx.parallel.boundary_slots).  The slots
 * are written, never added to, so left == right is safe. */
int fcx_set_atmos_shared(fcx_engine *e, double *shared, int32_t n_boundaries, int32_t stride,
                         int32_t left, int32_t right);
/* instead of fcx_set_atmos_shared: the engine allocates the [n_boundaries][fields] slots
 * itself (device memory, zeroed; stride = number of fcx_add_atmos_field fields).  Before
 * fcx_commit. */
int fcx_set_atmos_boundaries(fcx_engine *e, int32_t n_boundaries, int32_t left, int32_t right);
/* after the all-reduce of `shared`: boundary values -> out arrays, slots re-zeroed */
int fcx_atmos_finish(fcx_engine *e);
/* the accumulation of `phase` on its own (fcx_run runs it unless FCX_OPT_ATMOS_IN_RUN=0) */
int fcx_run_atmos(fcx_engine *e, int phase);

/* ---- the one collective: RCCL over xGMI ----
 * The boundary slots of all ranks are summed by ONE ncclAllReduce(sum, ncclFloat64) per
 * step, the exchange OASIS3-MCT performs on the oasis_put of the type-0 fields
 * (flux_calculator.F90:1015, create_namcouple.F90:92-98).  One communicator per rank (one
 * rank per GPU): rank 0 creates the unique id, the host broadcasts its
 * FCX_COMM_ID_BYTES bytes (MPI_Bcast in the Fortran host) and every rank creates its
 * communicator.  RCCL is loaded at run time (the process's own librccl.so if one is
 * already loaded, e.g. PyTorch's, else /opt/rocm's). */
#define FCX_COMM_ID_BYTES 128
typedef struct fcx_comm fcx_comm;
int fcx_comm_unique_id(void *id /* FCX_COMM_ID_BYTES */);
int fcx_comm_create(int device, int nranks, int rank, const void *id, fcx_comm **out);
int fcx_comm_destroy(fcx_comm *c);
/* sum-all-reduce of count doubles in place on a HIP stream (generic) */
int fcx_comm_allreduce_sum(fcx_comm *c, double *buf, size_t count, void *hip_stream);
/* attach: from now on fcx_run / fcx_step / fcx_run_atmos of the engine complete its
 * boundary slots themselves (all-reduce on the engine's stream, then fcx_atmos_finish);
 * every rank's engine must then run the same steps.  fcx_run_atmos after an fcx_run that
 * already exchanged issues no collective.  NULL detaches. */
int fcx_set_comm(fcx_engine *e, fcx_comm *c);
/* several engines of this rank (e.g. one per bottom-model variant) in ONE all-reduce of
 * sum(n_boundaries * stride) doubles over their slots in list order, on the first engine's
 * stream, then fcx_atmos_finish of each.  Regions that follow each other in list order in
 * one buffer are reduced in place, others through the communicator's scratch; the collective
 * is the same either way.  Call after their accumulation (fcx_run, or fcx_run_atmos).
 * Collective contract: every rank passes its engines in the same order with the same
 * n_boundaries and strides.  What is checked: by default, the FIRST exchange of each
 * signature a rank has not exchanged before on this communicator is preceded by a blocking
 * max-all-reduce of the signature, and ranks that disagree all return FCX_E_ARG -- this
 * catches a decomposition the ranks disagree on from the start, without a host wait per
 * step.  It cannot catch a rank that switches to a new engine list after exchanging while
 * another keeps an already agreed one (that rank skips the check, the collectives differ);
 * fcx_comm_verify(c, 1) runs the check before EVERY exchange (one 6-double all-reduce and a
 * host wait per exchange) for hosts that change their engine lists at run time.  An engine
 * already completed in this run (fcx_set_comm) takes part with zeros and is skipped; one
 * with no accumulation since its last exchange takes part with zeros and the call returns
 * FCX_E_STATE after the collective, so no rank is left waiting. */
int fcx_atmos_allreduce(fcx_comm *c, fcx_engine *const *engines, int n_engines);
/* 1: the signature agreement before every exchange of the communicator; 0 (default): before
 * the first exchange of each signature */
int fcx_comm_verify(fcx_comm *c, int every_exchange);

/* ---- exchange-grid -> model remaps ----
 * The SCRIP weight application OASIS3-MCT performs on the 'S' fields sent to a model
 * (remap files mappings/remap_<grid>_exchangegrid_to_<model>.nc): out[d] = sum over the
 * links k with dst[k] == d, in link order from 0.0, of w[k] * field[src[k]].  src: 0-based
 * cell of the field's grid on this rank; dst: 0-based cell of the target grid (n_dst cells,
 * e.g. the whole ocean grid).  With several ranks, every rank writes its partial sums of
 * all n_dst cells (0 where it has no link); an all-reduce (sum) of the output arrays over
 * the ranks completes them.  Run by fcx_run / fcx_step after the fluxes. */
int fcx_add_remap(fcx_engine *e, int64_t n_dst, int64_t n_links, const int32_t *src_cell,
                  const int32_t *dst_cell, const double *weight, int32_t *remap_id);
int fcx_add_remap_field(fcx_engine *e, int32_t remap_id, int phase, int surface_type, int grid,
                        int var, double *out, int flags);
/* after fcx_commit: the map's gather scatter (distinct 64-B field segments per link over a
 * sample of 256-destination blocks) and whether its launches gather packed records
 * (FCX_OPT_REMAP_PACK): 0 no, 1 packed by a packing pass, 2 the flux launch of the last
 * fcx_run / fcx_step wrote the records of one launch group of this remap (T=1 fluxes of
 * surface type 1; that group needs no packing pass -- a remap of more than 16 fields has
 * further groups, which pack their own).  Per-call runs do not change the answer. */
int fcx_remap_info(const fcx_engine *e, int32_t remap_id, double *scatter, int32_t *packed);

/* launch tuning of the fused cells kernel (defaults are the measured best on MI355X) */
enum fcx_option {
  FCX_OPT_CELLS_PER_THREAD = 1, /* 1 or 2 cells per lane (2: 16-B loads; default 2)       */
  FCX_OPT_MAX_BLOCKS = 2,       /* grid-stride cap in 256-thread blocks; 0 = no cap;
                                   -1 (default) = per kernel: 8192 for the flux pass, no
                                   cap for the T=1 pass with the fused accumulation       */
  FCX_OPT_NONTEMPORAL = 3,      /* non-temporal hint on streamed loads/stores (default 1) */
  FCX_OPT_SPECIALIZE = 4,       /* T=1 CCLM/MOM5/RCO specialised kernels (default 1)      */
  FCX_OPT_ATMOS_IN_RUN = 5,     /* fcx_run also runs the atmosphere accumulation (def. 1) */
  FCX_OPT_PIPELINE_CHUNKS = 7,  /* fcx_step of host-bound fields: H2D/compute/D2H overlap
                                   over this many cell chunks (default 8; 1 = sequential) */
  FCX_OPT_PIPELINE_MIN_CHUNK = 8, /* ... of at least this many cells (multiple of 1024;
                                   default 262144: smaller grids take the sequential step) */
  FCX_OPT_ZERO_COPY = 9,        /* fields used by the kernels in place through the host link:
                                   no mirrors, no copy calls (fcx_host_malloc arrays directly,
                                   caller heap arrays through the mapped staging arena).
                                   2 auto (default): when every grid is below
                                   2 x PIPELINE_MIN_CHUNK cells; 1: at any size; 0: never */
  FCX_OPT_LIB_SPANS = 19,       /* fcx_host_malloc arrays not used in place: device mirrors
                                   laid out like the host memory (one buffer per slab span), so
                                   arrays adjacent in host memory move as ONE copy per
                                   direction -- a host allocating its inputs, then its outputs,
                                   in the reference's order makes
                                   one or two uploads and one download per phase.  1 (default);
                                   0: one copy per array.  Applied at fcx_commit           */
  FCX_OPT_TIMING = 10,          /* record the events behind fcx_last_kernel_ms (default 0:
                                   two event records per run cost ~8 us on small grids) */
  FCX_OPT_HOST_STAGING = 15,    /* caller heap arrays (not fcx_host_malloc memory) reach
                                   their device mirrors through an engine-owned page-locked
                                   staging arena laid out like the mirrors: host threads copy
                                   the arrays into it, then ONE DMA per pool and direction
                                   (per chunk when pipelined), and back.  1 (default); 0:
                                   one runtime copy per array (pageable, staged by HIP).
                                   Nothing of the caller's memory is ever page-locked or
                                   mapped.  Applied at fcx_commit                          */
  FCX_OPT_HOST_THREADS = 16,    /* host threads of those copies (the calling thread
                                   included); 0 (default): min(16, OMP_NUM_THREADS if set,
                                   else the CPUs of the process affinity set -- divided by
                                   the node's local rank count when the rank is not pinned
                                   (OMPI_COMM_WORLD_LOCAL_SIZE, MPI_LOCALNRANKS,
                                   SLURM_NTASKS_PER_NODE or LOCAL_WORLD_SIZE)).  Under MPI,
                                   pin ranks or set this to each rank's core share        */
  FCX_OPT_DEFERRED_SCATTER = 18, /* staged downloads: 0 (default) fcx_download waits for the
                                   stream and fills the caller's heap arrays before it
                                   returns; 1: the host copies wait for the next
                                   fcx_synchronize (a host that overlaps engines)         */
  FCX_OPT_RETIRED_PIN_HOST = 6, /* retired options (version 3): accepted and ignored      */
  FCX_OPT_RETIRED_12 = 12,
  FCX_OPT_RETIRED_CARRY_HANDOFF = 14,
  FCX_OPT_ATMOS_HALO = 17,      /* fused accumulation of one surface type, launched over the
                                   whole grid, on a map whose segments are at most 9 cells:
                                   1 (default) halo tiles -- each wave also computes the
                                   head cells of the next tile for their products, so every
                                   segment completes inside the launch (no crossing records,
                                   no fix-up launch); 0: crossing records + fix-up launch  */
  FCX_OPT_REMAP_PACK = 13,      /* exchange -> model remaps: the fields of a launch packed
                                   cell-major into one record per exchange cell before the
                                   gather, so a link reads one record instead of nf
                                   scattered values.  2 auto (default): launches of >= 2
                                   fields; 1: always; 0: never (gather from the arrays).
                                   Applied at fcx_commit (scratch of cells x record)      */
  FCX_OPT_TILED_LAYOUT = 11     /* engine-owned mirrors tile-blocked (default 1): tiles of
                                   4096 cells, the read-only arrays' tiles interleaved in
                                   one pool and the written arrays' in another, so a wave's
                                   accesses fall in one contiguous region (+8-10 % streaming
                                   rate, components.flux_calculator_amd/bench/layout_probe.hip).
                                   Applied at fcx_commit when no field array is the caller's
                                   device memory or used in place (zero-copy) */
};
int fcx_set_option(fcx_engine *e, int option, int64_t value);

/* page-locked host memory owned by the library, mapped for the device at allocation: a
 * host that allocates its local_field arrays here (c_f_pointer in Fortran) gets the
 * zero-copy step on small grids (FCX_OPT_ZERO_COPY auto) and direct DMA on large ones,
 * without any registration of its own memory.  Free only after every engine using the
 * memory is destroyed.  No GPU work; callable before any engine exists. */
int fcx_host_malloc(size_t bytes, void **ptr);
int fcx_host_free(void *ptr);

/* device memory for hosts that keep fields resident in HBM (bind with FCX_MEM_DEVICE) */
int fcx_device_malloc(int device, size_t bytes, void **ptr);
int fcx_device_free(void *ptr);
/* synchronous copy; kind: 1 host->device, 2 device->host, 3 device->device */
int fcx_memcpy(void *dst, const void *src, size_t bytes, int kind);

#ifdef __cplusplus
}
#endif
#endif /* FCX_H */
