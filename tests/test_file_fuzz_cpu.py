"""The file-layer fuzz (tests/file_fuzz.py) on CPU, against the
asynchronous CPU stand-in for the device (tools/tsan/cpudev_async.c: a
worker thread per stream, the CPU oracle's conversions, every kernel access
checked against the device, pinned and registered ranges live when it
runs; test harness only, never part of the library).  All type pairs,
host and device buffers, vara / vars / varm, blocking and nonblocking,
CDF-5 and CDF-2: what it checks is the host logic -- where the file layer
puts bytes and how it orders the device's work -- with the device's
asynchrony emulated.  One sequence also runs with the host code and the
stand-in built under AddressSanitizer + UBSan.  The GPU twin
(tests/test_gpu_file_fuzz.py) runs the HIP kernels."""
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
from pnetcdf_amd import pncx
conv = OracleConv()
dev = file_fuzz.StandinDev(pncx.lib())
for seed in {seeds!r}:
    for fmt in {fmts!r}:
        c = file_fuzz.run({d!r} + "/fz_%d_%d.nc" % (seed, fmt), seed, conv, steps={steps}, fmt=fmt, dev=dev)
        print("seed", seed, "fmt", fmt, sorted(c.items()), flush=True)
print("fuzz ok")
"""


def _build(d, san):
    so = os.path.join(str(d), "libpncx_async%s.so" % ("_asan" if san else ""))
    c = os.path.join(ROOT, "pnetcdf_amd", "csrc")
    flags = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"] if san else []
    subprocess.run(["gcc", "-O1", "-g", "-fPIC", "-shared", *flags, "-I" + os.path.join(ROOT, "include"), "-I" + c,
                    os.path.join(c, "pncx_host.c"), os.path.join(c, "pncx_cdf.c"), os.path.join(c, "pncx_nc.c"),
                    os.path.join(c, "pncx_io.c"), os.path.join(ROOT, "tools", "tsan", "cpudev_async.c"),
                    os.path.join(ROOT, "oracle", "pncx_oracle.c"), "-o", so, "-lpthread", "-lm"],
                   check=True, capture_output=True, timeout=300)
    return so


@pytest.mark.parametrize("san", [False, True], ids=["plain", "asan-ubsan"])
def test_file_fuzz_async_standin(tmp_path, san):
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    env = dict(os.environ, PNCX_NO_TORCH="1")
    if san:
        lib = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
        if not os.path.isabs(lib) or not os.path.exists(lib):
            pytest.skip("libasan not available")
        env.update(LD_PRELOAD=lib, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env["PNCX_LIB_PATH"] = _build(tmp_path, san)
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)       # tmpfs: the appending-put paths
    d = os.path.join(shm, f"pncx_fz_cpu_{os.getpid()}_{int(san)}")
    os.makedirs(d, exist_ok=True)
    seeds, fmts = ([5], [2]) if san else ([11, 12, 13], [5, 2])
    try:
        out = subprocess.run([sys.executable, "-c", RUN.format(root=ROOT, seeds=seeds, fmts=fmts, d=d, steps=150)],
                             capture_output=True, text=True, env=env, timeout=900)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    assert out.returncode == 0, (out.stdout[-3000:], out.stderr[-5000:])
    assert "fuzz ok" in out.stdout
