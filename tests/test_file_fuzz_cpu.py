"""The file-layer fuzz (tests/file_fuzz.py) on CPU: the host sources built
against the synchronous CPU stand-in for the device (tools/tsan/
cpudev_stub.c, test harness only), so only same-type requests (byte swaps)
run; what this checks is the file layer's placement of bytes -- vara, vars,
varm with permuted and gapped imaps, records past numrecs, nonblocking
requests flushed together, a variable larger than a staging slot -- against
the model.  The GPU twin (tests/test_gpu_file_fuzz.py) runs every type
pair through the HIP kernels."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RUN = r"""
import sys
sys.path.insert(0, {root!r})
from tests import file_fuzz
from tests.converters import OracleConv
conv = OracleConv()
for seed in {seeds!r}:
    for fmt in (5, 2):
        c = file_fuzz.run({d!r} + "/fz_%d_%d.nc" % (seed, fmt), seed, conv, steps={steps}, fmt=fmt,
                          same_type=True, torch=None, imap=False)
        print("seed", seed, "fmt", fmt, sorted(c.items()), flush=True)
print("fuzz ok")
"""


@pytest.fixture(scope="module")
def cpudev_lib(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    d = tmp_path_factory.mktemp("cpudev")
    so = str(d / "libpncx_cpudev.so")
    c = os.path.join(ROOT, "pnetcdf_amd", "csrc")
    subprocess.run(["gcc", "-O1", "-g", "-fPIC", "-shared", "-I" + os.path.join(ROOT, "include"), "-I" + c,
                    os.path.join(c, "pncx_host.c"), os.path.join(c, "pncx_cdf.c"), os.path.join(c, "pncx_nc.c"),
                    os.path.join(c, "pncx_io.c"), os.path.join(ROOT, "tools", "tsan", "cpudev_stub.c"),
                    "-o", so, "-lpthread"], check=True, capture_output=True, timeout=300)
    return so


def test_file_fuzz_same_type_cpu(cpudev_lib, tmp_path):
    env = dict(os.environ, PNCX_LIB_PATH=cpudev_lib, PNCX_NO_TORCH="1")
    code = RUN.format(root=ROOT, seeds=[11, 12, 13], d=str(tmp_path), steps=120)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, (out.stdout[-3000:], out.stderr[-5000:])
    assert "fuzz ok" in out.stdout
