"""Helpers for the tests that drive the C programs of tests/mpi/ (programs
written against the reference's C interfaces and linked with this build's
libraries).  Test infrastructure only."""
import os
import shutil
import struct
import subprocess

import numpy as np

from pnetcdf_amd import nctypes as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPI_DIR = os.path.join(ROOT, "tests", "mpi")
MPIEXEC = "/opt/conda/bin/mpiexec"

# ncmpii_check.c mpi_type(i): the 11 numeric MPI itypes in enum pncx_itype
# order, MPI_CHAR, then two types with no conversion itype (MPI_BYTE,
# MPI_LONG_DOUBLE -> NC_EBADTYPE)
MPI_IDX_ITYPE = {i: i + 1 for i in range(11)}
MPI_IDX_ITYPE[11] = T.ITYPE_CHAR
MPI_UNKNOWN = (12, 13)
MPI_NAMES = ["MPI_SIGNED_CHAR", "MPI_UNSIGNED_CHAR", "MPI_SHORT", "MPI_UNSIGNED_SHORT", "MPI_INT",
             "MPI_UNSIGNED", "MPI_LONG", "MPI_FLOAT", "MPI_DOUBLE", "MPI_LONG_LONG_INT",
             "MPI_UNSIGNED_LONG_LONG", "MPI_CHAR", "MPI_BYTE", "MPI_LONG_DOUBLE"]
MPI_SIZE = [1, 1, 2, 2, 4, 4, 8, 4, 8, 8, 8, 1, 1, 16]


def exe(name):
    p = os.path.join(MPI_DIR, name)
    assert os.path.exists(p), f"{p} not built (run __graft_entry__.build())"
    return p


def run(args, nprocs=1, timeout=300, check=True, env=None):
    """Run a tests/mpi program, under mpiexec when nprocs > 1 (env: the
    environment to use instead of this process's)."""
    cmd = ([MPIEXEC, "-n", str(nprocs)] if nprocs > 1 else []) + list(args)
    env = dict(os.environ if env is None else env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=MPI_DIR)
    if check:
        assert r.returncode == 0, f"{cmd} -> {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return r


def have_mpiexec():
    return os.path.exists(MPIEXEC) and shutil.which("hydra_pmi_proxy", path="/opt/conda/bin") is not None


# ---------------------------------------------------------------- ncmpii_check
def case(op, cdf=5, xtype=0, mpi=0, nelems=0, fill=None, data=b""):
    f = (fill or b"") + b"\0" * 8
    return struct.pack("<6q", op, cdf, xtype, mpi, nelems, 1 if fill is not None else 0) + f[:8] + \
        struct.pack("<q", len(data)) + data


def read_results(path):
    b = open(path, "rb").read()
    out, p = [], 0
    while p < len(b):
        st, n = struct.unpack_from("<2q", b, p)
        p += 16
        out.append((st, b[p:p + n]))
        p += n
    return out
