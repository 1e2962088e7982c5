"""Host C code under ThreadSanitizer, on CPU (the
library's shared state across threads).  tools/tsan/run.sh builds the file
layer, the I/O pool and the host driver against a synchronous CPU stand-in
for the device (tools/tsan/cpudev_stub.c, a test harness that is never part
of the library) and runs tools/tsan/threads.c: six threads each create,
write (NC_BYTE, NC_CHAR, NC_INT from host and "device" buffers, NC_DOUBLE;
blocking and nonblocking), read back and reopen their own files, the shape
of the reference's test/testcases/tst_pthread.c, while a seventh churns the
file table.  Any data race report fails the run; the stand-in's launch
counts show the device paths (staging, piece events, batch completion) ran.

Round 6 found one race this way: the I/O layer's lazily read mmap mode
could be seen set before the page size it guards (pncx_io.c mmap_mode, now a
pthread_once).  The writers pass a barrier before their first data call so
that such first touches are unordered; with the old mmap_mode every case
here reports it (checked by reverting the fix).  STUB=nodev builds against
the no-device stub instead (the NC_BYTE / NC_CHAR paths only)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _have_tsan():
    if shutil.which("gcc") is None:
        return False
    lib = subprocess.run(["gcc", "-print-file-name=libtsan.so"], capture_output=True, text=True).stdout.strip()
    return os.path.isabs(lib) and os.path.exists(lib)


@pytest.mark.parametrize("env", [{"PNCX_STAGE_MB": "1"}, {"STUB": "nodev"}], ids=["1MiB-staging", "no-device"])
def test_host_code_tsan_clean(env):
    if not _have_tsan():
        pytest.skip("gcc or libtsan not available")
    e = dict(os.environ, NTHREADS="6", ITERS="2", **env)
    out = subprocess.run(["bash", os.path.join(ROOT, "tools", "tsan", "run.sh")], capture_output=True,
                         text=True, env=e, timeout=900)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-6000:])
    assert "ThreadSanitizer" not in out.stderr, out.stderr[-6000:]
    assert "threads ok 6 writers" in out.stdout, out.stdout


@pytest.mark.parametrize("san,dev", [("thread", "1"), ("address", "1")],
                         ids=["tsan-device-buffers", "asan-ubsan-device-buffers"])
def test_api_stack_sanitizers_clean(san, dev):
    """The whole host stack behind ncmpi_* (dispatcher, driver, ncmpii, file
    layer, I/O pool) under ThreadSanitizer: api_check's tst_pthread
    restatement (6 threads, the reference's 4 x 5 and 1 MiB records,
    collective and independent) and its 16-thread file-table churn, one MPI
    process with MPI_THREAD_MULTIPLE (tools/tsan/run_api.sh); then the
    single-threaded programs for configs 1, 4 and 5, the put_vara benchmark,
    define mode and the dispatcher's error returns.  With the dispatcher's
    mutex removed, the churn reports a race (checked by hand).  SAN=address
    runs the same programs under AddressSanitizer + UBSan."""
    mpi = os.environ.get("MPI_HOME", "/opt/conda")
    if not _have_tsan() or not os.path.exists(os.path.join(mpi, "lib", "libmpi.so")):
        pytest.skip("gcc/libtsan or MPI not available")
    out = subprocess.run(["bash", os.path.join(ROOT, "tools", "tsan", "run_api.sh"), dev], capture_output=True,
                         text=True, timeout=900, env=dict(os.environ, SAN=san))
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-6000:])
    assert "Sanitizer" not in out.stderr and "runtime error" not in out.stderr, out.stderr[-6000:]
    assert f"api {san} ok dev={dev}" in out.stdout, out.stdout[-2000:]
