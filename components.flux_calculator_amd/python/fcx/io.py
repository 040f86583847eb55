"""Readers of the exchange-grid files (flux_calculator_io.F90), for hosts that set the
engine up from the mapping files themselves.

* read_scrip_grid      -- read_scrip_grid_dimensions (io:28-107): grid size, centre lon/lat,
                          area, and the rank's range from the `task` vector
* read_regridding_matrix -- io:109-198: the COO links of the rank, 1-based local indices
* read_remapping       -- io:200-236: src/dst grid dimensions of an OASIS remapping file

NetCDF-3 files through scipy (no NetCDF library in this image; NetCDF-4/HDF5 files raise).
The semantics are restated from the Fortran; with no NetCDF library the reference itself
cannot run here, so these are "parity unpinned" (tests/test_io_readers.py exercises them on
files written here).
"""
import numpy as np


def _open(path):
    from scipy.io import netcdf_file

    with open(path, "rb") as fh:
        if fh.read(3) != b"CDF":
            raise ValueError(f"{path}: not a NetCDF-3 file (NetCDF-4/HDF5 needs a NetCDF library)")
    return netcdf_file(path, "r", mmap=False)


def read_scrip_grid(path, mype=0, num_tasks=1):
    """io:28-107 for one bottom model: {grid_size_global, lon, lat, area, grid_size,
    grid_offset}.  One task: the whole grid.  Several: the cells whose `task` entry equals
    mype; offset = first such cell - 1 (0-based); an empty task gets size 0, offset 0."""
    with _open(path) as f:
        n = f.dimensions["grid_size"]
        out = {"grid_size_global": int(n),
               "lon": np.array(f.variables["grid_center_lon"].data, dtype=np.float64),
               "lat": np.array(f.variables["grid_center_lat"].data, dtype=np.float64),
               "area": np.array(f.variables["grid_area"].data, dtype=np.float64)}
        if num_tasks == 1:
            out["grid_size"], out["grid_offset"] = int(n), 0
            return out
        task = np.array(f.variables["task"].data).astype(np.int64)
    hit = np.nonzero(task == mype)[0]
    if hit.size == 0:
        out["grid_size"], out["grid_offset"] = 0, 0
    else:
        out["grid_size"], out["grid_offset"] = int(hit.size), int(hit[0])
    return out


def read_regridding_matrix(path, src_grid_size, src_grid_offset, dst_grid_size, dst_grid_offset):
    """io:109-198: the links with dst in (dst_offset, dst_offset + dst_size], in file order,
    indices made local (1-based) by subtracting the offsets; a source outside the rank's
    range stops the run like the reference's MPI_Abort (io:188-193) -- here a ValueError.
    Returns (src_index int32, dst_index int32, weight float64), the arrays
    Engine(regrid={"matrices": {which: (src, dst, w)}}) takes."""
    with _open(path) as f:
        src = np.array(f.variables["src_address"].data).astype(np.int64)
        dst = np.array(f.variables["dst_address"].data).astype(np.int64)
        w = np.array(f.variables["remap_matrix"].data, dtype=np.float64)
    if w.ndim == 2:
        w = w[:, 0]  # remap_matrix(num_links, num_wgts): the first weight (io:155)
    keep = (dst > dst_grid_offset) & (dst <= dst_grid_offset + dst_grid_size)
    src_l = src[keep] - src_grid_offset
    dst_l = dst[keep] - dst_grid_offset
    bad = (src_l < 1) | (src_l > src_grid_size)
    if bad.any():
        raise ValueError(f"Regridding matrix did not match task decomposition in file {path} "
                         f"(link {int(np.nonzero(keep)[0][np.nonzero(bad)[0][0]]) + 1})")
    return (np.ascontiguousarray(src_l, dtype=np.int32), np.ascontiguousarray(dst_l, dtype=np.int32),
            np.ascontiguousarray(w[keep]))


def read_remapping(path):
    """io:200-236: (src_grid_dims, dst_grid_dims), a rank-1 grid padded with a 1."""
    with _open(path) as f:
        dims = []
        for side in ("src", "dst"):
            rank = int(f.dimensions[f"{side}_grid_rank"])
            d = [int(x) for x in np.array(f.variables[f"{side}_grid_dims"].data)[:rank]]
            if rank == 1:
                d.append(1)
            dims.append(tuple(d))
    return tuple(dims)


__all__ = ["read_scrip_grid", "read_regridding_matrix", "read_remapping"]
