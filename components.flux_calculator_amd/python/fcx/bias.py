"""Monthly bias corrections for a rank's cell range (bias_corrections.F90:170-245).

The reference reads `corrections/<name>-MM.nc` (MM = 01..12, bias:203-204) with
`nf90_get_var(..., corrections(i,j,:), (/grid_offset/), (/grid_size/))` (bias:220-222).
`grid_offset` is the 0-based first cell of the rank (io:75, 95) but NetCDF starts are
1-based: rank 0 (start 0) fails the read, and the month is silently zeroed (bias:223-227);
other ranks read one cell early.  `_FillValue` entries become 0
(bias:241); an unreadable file leaves the month at 0 (bias:207-218).

`window()` applies the intended slice `corr[month][offset : offset + size]` by default, or
the reference's behaviour with `reference_offset_quirk=True`, for comparisons against
output of the reference build.  The P5 semantics are inferred from the netcdf-fortran
documentation (no NetCDF library in this image): parity unpinned.

The result is month-major `[12][grid_size]`, the layout `Engine(corrections=(init_date,
array))` accepts directly (FCX_CORR_MONTH_MAJOR).
"""
import os

import numpy as np


def window(global_corr, grid_offset, grid_size, fill_value=None, reference_offset_quirk=False):
    """[12][grid_size] corrections of the cells [grid_offset, grid_offset + grid_size) from a
    month-major global field [12][n_global] (a month row may be None: file missing).
    fill_value: one value for all months, or a list of 12 (None entries: no replacement)."""
    out = np.zeros((12, grid_size))
    fills = list(fill_value) if isinstance(fill_value, (list, tuple)) else [fill_value] * 12
    for m in range(12):
        row = None if global_corr is None else global_corr[m]
        if row is None:
            continue  # bias:207-211: could not open -> correction stays 0
        row = np.asarray(row, dtype=np.float64)
        if reference_offset_quirk:
            start = grid_offset  # used as a 1-based NetCDF start
            if start < 1 or start - 1 + grid_size > row.shape[0]:
                continue  # nf90_get_var fails -> month zeroed (bias:223-227)
            vals = row[start - 1: start - 1 + grid_size]
        else:
            if grid_offset < 0 or grid_offset + grid_size > row.shape[0]:
                raise ValueError(f"cells [{grid_offset}, {grid_offset + grid_size}) outside the "
                                 f"{row.shape[0]}-cell correction field")
            vals = row[grid_offset: grid_offset + grid_size]
        vals = vals.copy()
        if fills[m] is not None:
            vals[vals == fills[m]] = 0.0  # bias:241
        out[m] = vals
    return out


def read_month_files(directory, name, fill_attr="_FillValue"):
    """The 12 global fields of corrections/<name>-MM.nc: ([12] rows or None, [12] fills).

    NetCDF-3 (classic / 64-bit offset) through scipy; a NetCDF-4/HDF5 file needs a NetCDF
    library this image lacks and raises.  A month whose file is missing, lacks the variable
    or lacks its _FillValue gives None: the reference leaves / sets it to 0 (bias:207-233)."""
    from scipy.io import netcdf_file

    rows, fills = [], []
    for m in range(1, 13):
        path = os.path.join(directory, f"{name}-{m:02d}.nc")
        if not os.path.exists(path):
            rows.append(None)
            fills.append(None)
            continue
        with open(path, "rb") as fh:
            magic = fh.read(4)
        if magic[:3] != b"CDF":
            raise ValueError(f"{path}: not a NetCDF-3 file (NetCDF-4/HDF5 needs a NetCDF library)")
        with netcdf_file(path, "r", mmap=False) as f:
            var = f.variables.get(name)
            if var is None or not hasattr(var, fill_attr):
                rows.append(None)  # bias:213-217 / 229-233: month stays / is set to 0
                fills.append(None)
                continue
            rows.append(np.array(var.data, dtype=np.float64).reshape(-1))
            fills.append(float(getattr(var, fill_attr)))
    return rows, fills


def read_bias_corrections(directory, name, grid_offset, grid_size, reference_offset_quirk=False):
    """initialize_bias_corrections for one correction: [12][grid_size] month-major."""
    rows, fills = read_month_files(directory, name)
    return window(rows, grid_offset, grid_size, fill_value=fills, reference_offset_quirk=reference_offset_quirk)


__all__ = ["window", "read_month_files", "read_bias_corrections"]
