"""pnetcdf_amd -- MI355X-native XDR byte-swap + NetCDF type-conversion path.

The product is the C-ABI library ``pnetcdf_amd/lib/libpncx.so``
(include/pncx.h) with hand-written HIP kernels for gfx950, plus the
reference-named MPI-typed shim ``libpncx_ncmpii.so`` (include/pncx_ncmpii.h).
This package is the Python host mirror used by tests and bench.
"""
from . import nctypes  # noqa: F401

__all__ = ["nctypes", "pncx"]
