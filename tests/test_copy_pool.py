"""The staging arena's host copy threads (fcx_copy_pool.h) on the CPU: a stress run of many
batches with random thread counts and sizes, compiled from the product header."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "copy_pool_stress.cpp")
INC = os.path.join(ROOT, "components.flux_calculator_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_copy_pool_stress(tmp_path):
    exe = str(tmp_path / "copy_pool_stress")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I" + INC, SRC, "-o", exe], check=True)
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "COPY_POOL_OK" in r.stdout
