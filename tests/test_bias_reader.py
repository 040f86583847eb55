"""Bias corrections of a rank's cell range (fcx.bias; bias_corrections.F90:170-245): the
intended window, the reference's 1-based-start quirk (P5: rank 0 zeroed, other ranks one
cell early), _FillValue -> 0, missing months -> 0, read from NetCDF-3 monthly files written
here with scipy (parity unpinned: no NetCDF library or reference output in this image)."""
import numpy as np
import pytest

from fcx.bias import read_bias_corrections, read_month_files, window
from fcx.parallel import apple_range


def global_field(n, seed=5):
    return np.random.default_rng(seed).normal(0, 1e-5, (12, n))


def test_intended_window_concatenates_to_the_global_field():
    g = global_field(1001)
    parts = [window(g, *apple_range(1001, r, 4)) for r in range(4)]
    np.testing.assert_array_equal(np.concatenate(parts, axis=1), g)


def test_reference_offset_quirk():
    g = global_field(100)
    # rank 0: start 0 is not a valid 1-based NetCDF start -> every month zeroed (bias:223-227)
    assert not window(g, 0, 25, reference_offset_quirk=True).any()
    # rank r > 0: start = grid_offset read as 1-based -> one cell early
    np.testing.assert_array_equal(window(g, 25, 25, reference_offset_quirk=True), g[:, 24:49])
    np.testing.assert_array_equal(window(g, 75, 25, reference_offset_quirk=True), g[:, 74:99])


def test_fill_values_and_missing_months_are_zero():
    g = global_field(50)
    g[3, 7] = -9999.0
    rows = [g[m] for m in range(12)]
    rows[5] = None
    w = window(rows, 0, 50, fill_value=-9999.0)
    assert w[3, 7] == 0.0 and not w[5].any()
    np.testing.assert_array_equal(w[4], g[4])


def test_read_netcdf3_month_files(tmp_path):
    from scipy.io import netcdf_file

    n = 64
    g = global_field(n, seed=9)
    g[0, 0] = 1e20
    for m in range(1, 13):
        if m == 7:
            continue  # a missing month
        with netcdf_file(str(tmp_path / f"mass_evap-{m:02d}.nc"), "w") as f:
            f.createDimension("grid_size", n)
            v = f.createVariable("mass_evap", "d", ("grid_size",))
            v[:] = g[m - 1]
            if m != 9:  # month 9 lacks _FillValue -> zeroed by the reference (bias:229-233)
                v._FillValue = np.float64(1e20)  # the variable's type, as NetCDF expects
    rows, fills = read_month_files(str(tmp_path), "mass_evap")
    assert rows[6] is None and rows[8] is None and fills[0] == 1e20
    c = read_bias_corrections(str(tmp_path), "mass_evap", 16, 32)
    assert c.shape == (12, 32)
    np.testing.assert_array_equal(c[1], g[1, 16:48])
    assert not c[6].any() and not c[8].any()
    c0 = read_bias_corrections(str(tmp_path), "mass_evap", 0, 16)
    assert c0[0, 0] == 0.0  # fill value replaced
    q = read_bias_corrections(str(tmp_path), "mass_evap", 16, 32, reference_offset_quirk=True)
    np.testing.assert_array_equal(q[1], g[1, 15:47])


def test_rejects_netcdf4(tmp_path):
    p = tmp_path / "mass_evap-01.nc"
    p.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(ValueError, match="NetCDF-3"):
        read_month_files(str(tmp_path), "mass_evap")
