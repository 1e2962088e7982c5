"""The integration patch applies to the
reference tree it was written against: a dry run of `patch -p1` over a copy
of the three files it touches.  CPU only; skipped where /root/reference is
absent (the GPU box)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCH = os.path.join(ROOT, "integration", "mi355x_one_round_trip.patch")
FILES = ["src/drivers/ncmpio/ncmpio_getput.m4", "src/drivers/ncmpio/ncmpio_i_getput.m4",
         "src/drivers/ncmpio/ncmpio_util.c"]


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("patch") is None,
                    reason="reference tree or patch(1) not available")
def test_patch_applies_to_reference(tmp_path):
    for f in FILES:
        dst = tmp_path / f
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(REF, f), dst)
    r = subprocess.run(["patch", "-p1", "--forward", "-i", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    got = (tmp_path / FILES[0]).read_text()
    assert "PNETCDF_MI355X_CONVERT" in got and "can_swap_in_place = 0" in got
