"""Exchange-grid file readers (fcx.io; flux_calculator_io.F90) on NetCDF-3 files written
here: the task-vector partition (io:68-104), the rank's regridding links with offset
correction and the decomposition check (io:109-198), the remapping dimensions
(io:200-236).  Parity unpinned: no NetCDF library or reference-produced files here."""
import numpy as np
import pytest

from fcx.io import read_regridding_matrix, read_remapping, read_scrip_grid
from fcx.parallel import task_range


def write_grid(path, task):
    from scipy.io import netcdf_file

    n = len(task)
    with netcdf_file(str(path), "w") as f:
        f.createDimension("grid_size", n)
        for name, vals in (("grid_center_lon", np.linspace(9, 31, n)), ("grid_center_lat", np.linspace(53.5, 66, n)),
                           ("grid_area", np.full(n, 2.5e7))):
            v = f.createVariable(name, "d", ("grid_size",))
            v[:] = vals
        t = f.createVariable("task", "i", ("grid_size",))
        t[:] = np.asarray(task, dtype=np.int32)


def write_links(path, src, dst, w, num_wgts=1):
    from scipy.io import netcdf_file

    with netcdf_file(str(path), "w") as f:
        f.createDimension("num_links", len(src))
        f.createDimension("num_wgts", num_wgts)
        a = f.createVariable("src_address", "i", ("num_links",))
        a[:] = np.asarray(src, dtype=np.int32)
        b = f.createVariable("dst_address", "i", ("num_links",))
        b[:] = np.asarray(dst, dtype=np.int32)
        m = f.createVariable("remap_matrix", "d", ("num_links", "num_wgts"))
        m[:] = np.repeat(np.asarray(w, dtype=np.float64)[:, None], num_wgts, axis=1)


def test_scrip_grid_task_ranges(tmp_path):
    task = [0] * 40 + [1] * 35 + [2] * 25
    write_grid(tmp_path / "t_grid.nc", task)
    g = read_scrip_grid(str(tmp_path / "t_grid.nc"))
    assert g["grid_size_global"] == 100 and (g["grid_size"], g["grid_offset"]) == (100, 0)
    assert g["lat"][0] == 53.5 and g["area"].shape == (100,)
    for r in range(4):  # rank 3 owns nothing: (0, 0) (io:101-104)
        g = read_scrip_grid(str(tmp_path / "t_grid.nc"), mype=r, num_tasks=4)
        assert (g["grid_offset"], g["grid_size"]) == task_range(np.array(task), r)


def test_regridding_links_of_a_rank(tmp_path):
    rng = np.random.default_rng(3)
    # global u->t links that respect a 2-way decomposition: t cells 1..50 | 51..100, u cells 1..48 | 49..90
    src, dst, w = [], [], []
    for (t0, t1), (u0, u1) in (((1, 50), (1, 48)), ((51, 100), (49, 90))):
        for d in range(t0, t1 + 1):
            for _ in range(3):
                src.append(rng.integers(u0, u1 + 1))
                dst.append(d)
                w.append(rng.uniform())
    order = rng.permutation(len(src))  # file order is arbitrary; the reader keeps it
    src, dst, w = np.array(src)[order], np.array(dst)[order], np.array(w)[order]
    write_links(tmp_path / "regrid_u_to_t.nc", src, dst, w, num_wgts=3)
    s1, d1, w1 = read_regridding_matrix(str(tmp_path / "regrid_u_to_t.nc"), 42, 48, 50, 50)
    keep = (dst > 50) & (dst <= 100)
    np.testing.assert_array_equal(d1, dst[keep] - 50)
    np.testing.assert_array_equal(s1, src[keep] - 48)
    np.testing.assert_array_equal(w1, w[keep])
    assert d1.dtype == np.int32 and s1.min() >= 1 and s1.max() <= 42
    # a decomposition the links do not match: the reference aborts (io:188-193)
    with pytest.raises(ValueError, match="did not match task decomposition"):
        read_regridding_matrix(str(tmp_path / "regrid_u_to_t.nc"), 40, 50, 50, 50)


def test_remapping_dimensions(tmp_path):
    from scipy.io import netcdf_file

    p = tmp_path / "remap.nc"
    with netcdf_file(str(p), "w") as f:
        f.createDimension("src_grid_rank", 1)
        f.createDimension("dst_grid_rank", 2)
        a = f.createVariable("src_grid_dims", "i", ("src_grid_rank",))
        a[:] = [12345]
        b = f.createVariable("dst_grid_dims", "i", ("dst_grid_rank",))
        b[:] = [94, 90]
    assert read_remapping(str(p)) == ((12345, 1), (94, 90))
