"""Set-up from flux_calculator.nml (fcx.namelist, fcx.setup) and --generate_namcouple
(fcx.namcouple), CPU only.

Each expectation is derived by hand from the reference statements cited next to it; the
reference set-up itself needs MPI, OASIS3-MCT and NetCDF and cannot run in this image
(parity unpinned against a reference run)."""
import numpy as np
import pytest

import namelists
from fcx.namcouple import counterpart, create_namcouple, header, mapping_file
from fcx.namelist import read_correctionsctl, read_input
from fcx.setup import SetupError, count_bottom_models, find_bottom_model, setup_from_namelist

GRIDS = (301, 299, 311)


# ---------------------------------------------------------------------------- namelist
def test_namelist_sequence_sections_nulls_repeats_truncation():
    v = read_input("""
    &input
      timestep = 600, num_timesteps= 24 ! comment, with 'quote
      name_bottom_model(1) = 'MOM5_Baltic', letter_bottom_model = 'M'
      name_bottom_var_t(1,1,:) = 'TSUR', 'FICE' 'ALBE',, 'FARE'
      val_bottom_var_t(1,2,2) = -2.0d20
      send_uniform_t(1,1:3) = 2*.true.
      send_to_atmos_t = F, , .t.
      which_flux_momentum(1,1) = 'MOM5', 'RCO'
      name_send_t = 3*'MEVA', 2*, 'HLATXX'
      name_atmos_model = "it's"
    /""")
    assert (v["timestep"], v["num_timesteps"]) == (600, 24)
    assert list(v["name_bottom_var_t"][0, 0, :6]) == ["TSUR", "FICE", "ALBE", "none", "FARE", "none"]
    assert v["val_bottom_var_t"][0, 1, 1] == -2.0e20 and v["val_bottom_var_t"][0, 1, 0] == -1.0e20
    assert list(v["send_uniform_t"][0, :4]) == [True, True, False, False]
    assert list(v["send_to_atmos_t"][:4]) == [False, True, True, True]  # null keeps the default
    # a scalar start continues in array-element order: (1,1) then (2,1)
    assert v["which_flux_momentum"][0, 0] == "MOM5" and v["which_flux_momentum"][1, 0] == "RCO"
    assert list(v["name_send_t"][:7]) == ["MEVA"] * 3 + ["none"] * 2 + ["HLAT", "none"]  # len=4
    assert v["name_atmos_model"] == "it's"
    c = read_correctionsctl(namelists.MOM5_BALTIC)
    assert c["init_date"] == 20000101 and c["lcorrections"][0] is True


@pytest.mark.parametrize("text, msg", [
    ("&input nonsense = 1 /", "unknown variable"),
    ("&input timestep = 1, 2 /", "too many values"),
    ("&input letter_bottom_model(11) = 'X' /", "out of bounds"),
    ("&input timestep = 'x' /", "character value"),
    ("&other x = 1 /", "not found"),
])
def test_namelist_errors(text, msg):
    with pytest.raises(ValueError, match=msg):
        read_input(text)


# --------------------------------------------------------------------- who am I (F90:262-310)
def test_bottom_model_walk_and_gaps():
    v = read_input("&input name_bottom_model = 'A1', 'B2', letter_bottom_model = 'X', 'Y', "
                   "num_tasks_per_model = 2, 3 /")
    assert count_bottom_models(v) == 2
    assert [find_bottom_model(v, r, 2) for r in range(5)] == [1, 1, 2, 2, 2]
    with pytest.raises(SetupError, match="Too many MPI instances"):
        find_bottom_model(v, 5, 2)
    gap = read_input("&input name_bottom_model(2) = 'B2' /")
    with pytest.raises(SetupError, match="must not contain gaps"):
        count_bottom_models(gap)
    reserved = read_input("&input name_bottom_model = 'B', letter_bottom_model = 'S', num_tasks_per_model = 1 /")
    with pytest.raises(SetupError, match="reserved"):
        setup_from_namelist("&input name_bottom_model = 'B', letter_bottom_model = 'S' /", grid_size=GRIDS)
    assert reserved["letter_bottom_model"][0] == "S"


# ---------------------------------------------------------------- STEP 1.4-1.7 on MOM5_BALTIC
@pytest.fixture(scope="module")
def mom5():
    return setup_from_namelist(namelists.MOM5_BALTIC, grid_size=GRIDS)


def test_received_fields(mom5):
    s = mom5
    assert s.num_surface_types == 2 and s.my_bottom_letter == "M"
    # bottom types in order (constants and -2e20 entries are not received), then atmosphere
    assert [f.name for f in s.input_field] == [
        "RMTSUR01", "RMFARE01", "RMFICE01", "RMALBE01", "RMCMOI01", "RMCHEA01", "RMCMOM01",
        "RMTSUR02", "RMFARE02", "RMALBE02", "RMCMOI02", "RMCHEA02",
        "RAPATM00", "RAPSUR00", "RAQATM00", "RATATM00", "RAUATM00", "RAVATM00"]
    early = {f.name for f in s.input_field if f.early}  # basic:154-156
    assert early == {"RMTSUR01", "RMFARE01", "RMALBE01", "RMCMOI01", "RMCHEA01", "RMCMOM01",
                     "RMTSUR02", "RMFARE02", "RMALBE02", "RMCMOI02", "RMCHEA02"}
    lf = s.local_field
    # atmosphere fields: one array, every surface type points at it (distribute_input_field)
    for v in ("PATM", "TATM", "UATM"):
        assert lf[(1, 1, v)] is lf[(0, 1, v)] and lf[(2, 1, v)] is lf[(0, 1, v)]
    # constant value (init_localvar) and -2e20 (type-1 pointer)
    assert np.all(lf[(2, 1, "FICE")] == 1.0)
    assert lf[(2, 1, "CMOM")] is lf[(1, 1, "CMOM")]
    assert (2, 1, "CMOM") in lf.allocated  # pointer assignment keeps the flag (basic:352)


def test_regridding_prepared_for_received_fields(mom5):
    lf = mom5.local_field
    for v in ("TSUR", "FICE", "CMOM", "PSUR", "TATM", "UATM", "VATM"):
        assert lf.put_to[(1, 1, v)] == 2 | 4  # t -> u and t -> v (basic:419-458)
        for g in (2, 3):
            assert (1, g, v) in lf.allocated
    # only received fields are regridded: the ice CMOM / FICE (not received) are not
    assert (2, 2, "CMOM") not in lf.field and (2, 2, "FICE") not in lf.field


def test_prepared_outputs_and_copy(mom5):
    lf = mom5.local_field
    for v, g in (("QSUR", 1), ("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1)):
        for s in (1, 2):
            assert (s, g, v) in lf.allocated
    assert (1, 2, "QSUR") in lf.allocated and (2, 2, "QSUR") not in lf.field  # 'none' on u for ice
    assert lf[(2, 2, "UMOM")] is lf[(1, 2, "UMOM")]  # 'copy' (prepare:36-38)
    assert lf[(2, 3, "VMOM")] is lf[(1, 3, "VMOM")]


def test_sent_fields_aliases_defaults_and_averages(mom5):
    s = mom5
    lf = s.local_field
    assert [f.name for f in s.output_field] == [
        "SAMEVA00", "SMMEVA01", "SMMEVA02", "SAUMOM00", "SMUMOM01", "SAVMOM00", "SMVMOM01",
        "SAHLAT00", "SMHLAT01", "SMHLAT02", "SAHSEN00", "SMHSEN01", "SMHSEN02",
        "SARBBR00", "SMRBBR01", "SATSUR00", "SARLWU00", "SMRLWU01", "SMRLWU02"]
    # uniform sends alias type 0 to the first type that has the flux, flag left unset
    assert lf[(0, 1, "RBBR")] is lf[(1, 1, "RBBR")] and (0, 1, "RBBR") not in lf.allocated
    assert lf[(0, 2, "UMOM")] is lf[(1, 2, "UMOM")]
    # non-uniform type-0 sends get their own array
    assert (0, 1, "MEVA") in lf.allocated and lf[(0, 1, "MEVA")] is not lf[(1, 1, "MEVA")]
    # TSUR to the atmosphere only: the t grid passes uniform=.FALSE. (F90:698-699)
    assert (0, 1, "TSUR") in lf.allocated
    # RLWU is computed nowhere: default-valued arrays and the reference's warnings
    for t in (0, 1, 2):
        assert np.all(lf[(t, 1, "RLWU")] == -5.0)
    assert sum("WARNING: Flux RLWU" in m for m in s.log) == 3
    # the put loops average type-0 fields with their own array when type 2 exists
    assert s.averages() == [(1, 1, "TSUR"), (2, 1, "MEVA"), (2, 1, "HLAT"), (2, 1, "HSEN"), (2, 1, "RLWU")]
    assert s.methods["which_flux_momentum"] == ["MOM5", "copy"]


def test_regrid_setup_second_bottom_model():
    s = setup_from_namelist(namelists.CCLM_REGRID, mype=1, grid_size=GRIDS)
    assert s.my_bottom_model == 2 and s.my_bottom_letter == "M" and s.num_surface_types == 1
    lf = s.local_field
    assert lf.put_to[(1, 1, "TSUR")] == 6 and lf.put_to[(1, 2, "UMOM")] == 1 and lf.put_to[(1, 3, "VMOM")] == 1
    assert (1, 1, "UMOM") in lf.allocated and (1, 1, "VMOM") in lf.allocated
    assert [f.name for f in s.output_field] == [
        "SAMEVA00", "SMMEVA01", "SAHLAT00", "SMHLAT01", "SAHSEN00", "SMHSEN01",
        "SARBBR00", "SMRBBR01", "SAUMOM00", "SMUMOM01", "SAVMOM00", "SMVMOM01"]
    assert lf[(0, 1, "UMOM")] is lf[(1, 1, "UMOM")]
    assert s.averages() == []  # one surface type: never averaged


@pytest.mark.parametrize("patch, msg", [
    ("which_flux_mass_evap(1,1) = 'XYZ'", "Method XYZ"),
    # MOM5 sensible heat needs CHEA: drop it from the water type's inputs
    ("name_bottom_var_t(1,1,6) = 'none'", "lacking the following variables:  CHEA"),
    # HLAT 'copy' checks type 1's HSEN (prepare:126), which is prepared only after HLAT
    # (F90:609-619): the reference rejects it unless HSEN is received
    ("which_flux_heat_latent(1,2) = 'copy'", "HLAT for surface_type=1"),
    ("which_flux_heat_latent(1,2) = 'copy'\n  name_bottom_var_t(1,1,8) = 'HSEN'", None),
    # a non-uniform momentum send needs FARE on the u grid
    ("send_uniform_u(1,1) = F", "fractional area"),
    # regridding onto a slot that is allocated already
    ("name_bottom_var_u(1,1,1) = 'TSUR'", "already exists on that grid"),
])
def test_setup_errors(patch, msg):
    end = "  send_uniform_v(1,1) = T\n/"  # patches go last: a later assignment wins
    assert end in namelists.MOM5_BALTIC
    text = namelists.MOM5_BALTIC.replace(end, f"  send_uniform_v(1,1) = T\n  {patch}\n/", 1)
    if msg is None:
        s = setup_from_namelist(text, grid_size=GRIDS)
        assert s.local_field[(2, 1, "HLAT")] is s.local_field[(1, 1, "HLAT")]  # the copy alias
        return
    with pytest.raises(SetupError, match=msg):
        setup_from_namelist(text, grid_size=GRIDS)


def test_single_type_atmosphere_only_send_is_left_unwritten():
    """T = 1, type-0 send on t to the atmosphere only: uniform=.FALSE. allocates a type-0
    array that no average ever fills (the put loops need local_field(2), F90:1003-1004)."""
    text = namelists.CCLM_REGRID.replace("send_uniform_t(2,1:6) = 6*.true.", "send_to_bottom_t(2,1) = F")
    s = setup_from_namelist(text, mype=1, grid_size=GRIDS)
    lf = s.local_field
    assert (0, 1, "MEVA") in lf.allocated and lf[(0, 1, "MEVA")] is not lf[(1, 1, "MEVA")]
    assert (2, 1, "MEVA") not in s.averages()


# ------------------------------------------------------------------------------ namcouple
def _dims(mf):
    return ((110, 120), (4000, 1)) if "exchangegrid_to" in mf else ((300, 1), (50, 60))


def test_namcouple_header_and_entries(mom5):
    text = create_namcouple(mom5, remapping_dims=_dims)
    lines = text.splitlines()
    n_in, n_out = len(mom5.input_field), len(mom5.output_field)
    assert lines[:14] == header(n_in, n_out, 600, 3)
    assert lines[1] == "  $NFIELDS" and lines[2].split() == [str(n_in + n_out)]
    assert lines[6].split() == ["1800"] and lines[10] == " 0 1"
    body = lines[14:]
    assert len(body) == 7 * (n_in + n_out)
    # sent fields first, then received ones, 7 lines each
    first = [body[7 * k].split()[0 if k < n_out else 1] for k in range(n_in + n_out)]
    assert first == [f.name for f in mom5.output_field] + [f.name for f in mom5.input_field]
    e = body[:7]  # SAMEVA00 to the atmosphere
    assert e[0] == "SAMEVA00 ARMEVA00 1 600 2 restart_flc_MEVA_CCLM_Eurocordex.nc EXPORTED"
    assert e[1].split() == ["110", "120", "4000", "1", "___", "___", "LAG=0"]
    assert e[2:] == [" R 0 R 0", " LOCTRANS MAPPING", " INSTANT",
                     " mappings/remap_t_grid_exchangegrid_to_CCLM_Eurocordex.nc", " ####"]
    k = [f.name for f in mom5.input_field].index("RMTSUR02")
    e = body[7 * (n_out + k): 7 * (n_out + k) + 7]  # a received bottom field
    assert e[0] == "MSTSUR02 RMTSUR02 1 600 2 restart_flc_TSUR_MOM5_Baltic.nc EXPORTED"
    assert e[1].split()[:4] == ["300", "1", "50", "60"]
    assert e[5] == " mappings/remap_t_grid_MOM5_Baltic_to_exchangegrid.nc"
    k = [f.name for f in mom5.output_field].index("SMUMOM01")
    assert body[7 * k + 5] == " mappings/remap_u_grid_exchangegrid_to_MOM5_Baltic.nc"


def test_namcouple_verbosity_debug_and_names():
    s = setup_from_namelist(namelists.CCLM_REGRID, mype=1, grid_size=GRIDS)
    text = create_namcouple(s, remapping_dims=_dims, debug_build=True)
    lines = text.splitlines()
    assert lines[10] == " 1 1"  # IOW_ESM_DEBUG
    assert lines[14].endswith(" EXPOUT")  # verbosity_level = 2
    assert counterpart("RAPATM00") == "ASPATM00" and counterpart("SMMEVA01") == "MRMEVA01"
    assert mapping_file("RAPATM00", 2, "CCLM") == "mappings/remap_u_grid_CCLM_to_exchangegrid.nc"


def test_namcouple_reads_remapping_files(tmp_path, mom5):
    """Default path: the dims come from the mapping files (read_remapping, io:200-236)."""
    from scipy.io import netcdf_file

    mf = set()
    for f in mom5.output_field + mom5.input_field:
        from fcx.namcouple import model_name
        nml = mom5.nml
        mf.add(mapping_file(f.name, f.which_grid, model_name(f.name, nml["name_atmos_model"],
                                                             nml["name_bottom_model"], nml["letter_bottom_model"])))
    (tmp_path / "mappings").mkdir()
    for k, name in enumerate(sorted(mf)):
        with netcdf_file(str(tmp_path / name), "w") as nc:
            nc.createDimension("src_grid_rank", 1)
            nc.createDimension("dst_grid_rank", 2)
            v = nc.createVariable("src_grid_dims", "i", ("src_grid_rank",))
            v[:] = [1000 + k]
            v = nc.createVariable("dst_grid_dims", "i", ("dst_grid_rank",))
            v[:] = [20 + k, 30]
    text = create_namcouple(mom5, directory=str(tmp_path))
    lines = text.splitlines()[14:]
    for k in range(len(lines) // 7):
        ent = lines[7 * k: 7 * k + 7]
        j = sorted(mf).index(ent[5].strip())
        assert ent[1].split()[:4] == [str(1000 + j), "1", str(20 + j), "30"]


# ------------------------------------------------------------- the time loop on the oracle
def test_time_loop_on_the_oracle_puts_reference_averages():
    """fcx.driver over the C oracle (no GPU): every put is finite, and a type-0 put that
    the put loop averages is sum_j FARE_j * flux_j in type order from 0.0 (calc:376-383)."""
    import oracle_lib
    from fcx import driver
    from fcx.synthetic import SyntheticCoupler

    s = setup_from_namelist(namelists.MOM5_BALTIC, grid_size=GRIDS)
    c = SyntheticCoupler.for_setup(s)
    driver.run(s, oracle_lib.OracleEngine(s, regrid=namelists.regrid_matrices(GRIDS)), c)
    assert len(c.sent) == 3 * len(s.output_field)
    assert all(np.all(np.isfinite(v)) for v in c.sent.values())
    t = 1200
    fare = [c._values(1, t)[1][j]["FARE"] for j in range(2)]
    for name in ("HLAT", "HSEN", "MEVA"):
        want = (0.0 + c.sent[(f"SM{name}01", t)] * fare[0]) + c.sent[(f"SM{name}02", t)] * fare[1]
        np.testing.assert_array_equal(c.sent[(f"SA{name}00", t)], want, err_msg=name)
    # uniform RBBR: the atmosphere gets type 1's array itself
    np.testing.assert_array_equal(c.sent[("SARBBR00", t)], c.sent[("SMRBBR01", t)])
