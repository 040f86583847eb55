"""`flux_calculator --generate_namcouple`: the OASIS3-MCT namcouple of one flux_calculator
set-up (flux_calculator_create_namcouple.F90:15-155, called at flux_calculator.F90:771-777).

    text = create_namcouple(setup, remapping_dims)        # or write_namcouple(path, ...)

One entry per sent field, then one per received field, in the set-up's list order:
  * the model a field talks to: name(2:2) == 'A' -> name_atmos_model, else the bottom model
    whose letter_bottom_model equals name(2:2) (create_namcouple:68-78; the name is a
    CHARACTER(len=32) there, so longer model names are cut to 32 characters);
  * the counterpart name swaps the first two letters' roles: RMTSUR01 <-> MSTSUR01
    (create_namcouple:103-106);
  * the mapping file mappings/remap_<grid>_<model>_to_exchangegrid.nc for received fields
    and mappings/remap_<grid>_exchangegrid_to_<model>.nc for sent ones (:91-98), whose
    src/dst grid dims (read_remapping, io:200-236; rank 1 padded with 1) go on the entry's
    second line;
  * EXPOUT when verbosity_level > 1, else EXPORTED (:62-66); $NLOGPRT '1 1' for an
    IOW_ESM_DEBUG build, else '0 1' (:29-34).
Records written with WRITE(unit,*) are list-directed; they are rendered here the way the
Intel and GNU runtimes do (a leading blank, default integers in 12 columns, a blank
between a number and a following string).  OASIS reads the file as whitespace-separated
tokens, and tests/test_setup_namcouple.py checks every line's tokens against the
statements of create_namcouple.F90 (parity unpinned against a reference run: the
reference needs MPI and NetCDF to run at all).

`remapping_dims(mapping_file) -> ((src_nx, src_ny), (dst_nx, dst_ny))`; the default reads
the NetCDF-3 file relative to `directory` with fcx.io.read_remapping.
"""
import os

from .basic import GRID_NAME, MAX_BOTTOM_MODELS

VERBOSITY_LEVEL_STANDARD = 1  # basic:70-72


def _ld(*items):
    """One list-directed record (WRITE(unit,*) items)."""
    out, prev_num = "", False
    for it in items:
        if isinstance(it, bool) or not isinstance(it, int):
            s = str(it)
            out += (" " if out == "" or prev_num else "") + s
            prev_num = False
        else:
            out += f"{it:12d}"
            prev_num = True
    return out


def header(num_input_fields, num_output_fields, timestep, num_timesteps, debug_build=False):
    """write_header (create_namcouple:15-39)."""
    return [
        _ld("####################################################################"),
        _ld(" $NFIELDS"),
        _ld(num_input_fields + num_output_fields),
        _ld(" $END"),
        _ld("############################################"),
        _ld(" $RUNTIME"),
        _ld(timestep * num_timesteps),
        _ld(" $END"),
        _ld("############################################"),
        _ld(" $NLOGPRT"),
        _ld("1 1" if debug_build else "0 1"),
        _ld(" $END"),
        _ld("############################################"),
        _ld(" $STRINGS"),
    ]


def model_name(io_name, name_atmos_model, name_bottom_model, letter_bottom_model):
    """create_namcouple:68-78, CHARACTER(len=32) my_model_name."""
    if io_name[1] == "A":
        name = name_atmos_model
    else:
        for i in range(MAX_BOTTOM_MODELS):
            if i < len(letter_bottom_model) and io_name[1] == letter_bottom_model[i]:
                name = name_bottom_model[i]
                break
        else:
            raise ValueError(f"{io_name}: no bottom model has the letter {io_name[1]!r}")
    return name[:32].rstrip()


def mapping_file(io_name, which_grid, my_model_name):
    """create_namcouple:91-98 (CHARACTER(len=128))."""
    grid = GRID_NAME[which_grid - 1]
    if io_name[0] == "R":
        f = f"mappings/remap_{grid}_{my_model_name}_to_exchangegrid.nc"
    else:
        f = f"mappings/remap_{grid}_exchangegrid_to_{my_model_name}.nc"
    return f[:128]


def counterpart(io_name):
    """create_namcouple:103-106: name(2:2) // other_io // name(3:8)."""
    other = "S" if io_name[0] == "R" else "R"
    return io_name[1] + other + io_name[2:]


def entry(io_field, name_atmos_model, name_bottom_model, letter_bottom_model, timestep,
          remapping_dims, verbosity_level=VERBOSITY_LEVEL_STANDARD):
    """create_namcouple_entry (create_namcouple:41-123): the entry's 7 lines."""
    export = "EXPOUT" if verbosity_level > VERBOSITY_LEVEL_STANDARD else "EXPORTED"
    name = io_field.name
    model = model_name(name, name_atmos_model, name_bottom_model, letter_bottom_model)
    mf = mapping_file(name, io_field.which_grid, model)
    (s0, s1), (d0, d1) = remapping_dims(mf)
    other = counterpart(name)
    first, second = (other, name) if name[0] == "R" else (name, other)
    tail = f" 2 restart_flc_{name[2:6].rstrip()}_{model}.nc "
    return [
        f"{first:<8s} {second:<8s} 1 {timestep}{tail}{export}",  # '(A, A, A, A, I0, A, A)'
        _ld(int(s0), int(s1), int(d0), int(d1), "___ ___ LAG=0"),
        _ld("R 0 R 0"),
        _ld("LOCTRANS MAPPING"),
        _ld("INSTANT"),
        _ld(mf.rstrip()),
        _ld("####"),
    ]


def _file_dims(directory):
    from .io import read_remapping

    return lambda mf: read_remapping(os.path.join(directory, mf))


def create_namcouple(setup, remapping_dims=None, directory=".", debug_build=False):
    """create_namcouple (create_namcouple:125-155) for a fcx.setup.FluxCalculatorSetup;
    returns the file's text."""
    nml = setup.nml
    dims = remapping_dims or _file_dims(directory)
    lines = header(len(setup.input_field), len(setup.output_field), nml["timestep"],
                   nml["num_timesteps"], debug_build)
    for f in list(setup.output_field) + list(setup.input_field):
        lines += entry(f, nml["name_atmos_model"], nml["name_bottom_model"], nml["letter_bottom_model"],
                       nml["timestep"], dims, nml["verbosity_level"])
    return "\n".join(lines) + "\n"


def write_namcouple(path, setup, remapping_dims=None, directory=".", debug_build=False):
    text = create_namcouple(setup, remapping_dims, directory, debug_build)
    with open(path, "w") as f:
        f.write(text)
    return text


__all__ = ["header", "entry", "model_name", "mapping_file", "counterpart", "create_namcouple",
           "write_namcouple"]
