"""The file-layer fuzz (tests/file_fuzz.py) on the GPU: seeded sequences of
blocking and nonblocking puts and gets -- vara, vars, varm with permuted
and gapped imaps, host numpy and hipMalloc'ed torch buffers, every internal
type against every external type of the format, values sometimes out of
range -- checked request by request against the oracle-driven model, and
the file's bytes after close.  CDF-5 (all ten external types) and CDF-1 /
CDF-2 (the classic five)."""
import os

import pytest

from tests import file_fuzz
from tests.converters import OracleConv

pytestmark = [
    pytest.mark.gpu,
    # Opt-in (PNCX_GPU_FUZZ=1): with copy-engine staging the fuzz still hits
    # a rare illegal-address fault (about 1 in 700 sequences, kernel not yet
    # identified, DESIGN §0 "late" and §11), and a fault in a shared test run
    # takes the device down for every later test; tools/fuzz_repeat.py runs it
    # on its own.  The CPU twin (tests/test_file_fuzz_cpu.py) always runs.
    pytest.mark.skipif(not os.environ.get("PNCX_GPU_FUZZ"), reason="GPU file fuzz is opt-in (PNCX_GPU_FUZZ=1)"),
]

SHM = "/dev/shm" if os.path.isdir("/dev/shm") else None


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


@pytest.mark.parametrize("seed,fmt", [(1, 5), (2, 5), (3, 5), (4, 5), (5, 1), (6, 2), (7, 5), (8, 2)])
def test_file_fuzz(gpu, tmp_path, seed, fmt):
    d = SHM or str(tmp_path)
    path = os.path.join(d, f"pncx_fuzz_{os.getpid()}_{seed}.nc")
    try:
        os.makedirs("gpurun_out", exist_ok=True)
        counts = file_fuzz.run(path, seed, OracleConv(), steps=150, fmt=fmt, torch=gpu,
                               log_path=f"gpurun_out/fuzz_{seed}_{fmt}.log")
    finally:
        if os.path.exists(path):
            os.unlink(path)
    print(seed, fmt, sorted(counts.items()))
    assert counts.get("put", 0) + counts.get("iput", 0) > 30
