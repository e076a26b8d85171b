"""The light grid on the CPU (no GPU needed): tests/native/grid_walk_check.cpp
builds host/bvh.cpp's grid and runs light_grid.hpp's cell walk -- the f64
instance the parity kernels run -- over random light sets (the scenes::simple
field with its large light, random sizes and negative radii, coincident
centres and zero radii, a huge light, non-finite entries) at 1/16 to 16 cells
per light, with on-surface, open, grazing and axis-aligned rays: every light
a ray hits must be counted exactly once, and none twice."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_grid_walk_counts_every_hit_light_once(tmp_path):
    exe = str(tmp_path / "grid_walk_check")
    subprocess.run([HIPCC, "-x", "hip", "--cuda-host-only", "-O2", "-std=c++17", "-I", CSRC,
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "native", "grid_walk_check.cpp"),
                    "-x", "c++", os.path.join(CSRC, "host", "bvh.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 wrong" in r.stdout
