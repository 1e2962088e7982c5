"""Host C code (header codec, file layer, I/O pool, dispatch) under
AddressSanitizer + UndefinedBehaviorSanitizer with leak checking, on CPU:
tools/asan/run.sh builds the C sources with a no-device shim and runs the
reference fixtures, the no-conversion data paths and a mutation fuzz of the
header decoder (corrupt files must fail cleanly, never touch memory they do
not own)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_asan_clean():
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(libasan) or not os.path.exists(libasan):
        pytest.skip("libasan not available")
    env = dict(os.environ, FUZZ_ROUNDS="800")
    out = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan", "run.sh")], capture_output=True,
                         text=True, env=env, timeout=600)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-4000:])
    assert "fuzz ok 800 mutants" in out.stdout
