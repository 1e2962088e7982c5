"""bench.py on the GPU at small sizes: the headline workload's check must
really check (every element), and the N > 1 path -- launcher, rank
reductions, distinct-device report, gather checksums -- runs as two ranks on
the one GPU of the box over gloo (PNCX_DIST_BACKEND=gloo: the rehearsal
mode that puts every rank on GPU 0 and says so in the line)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = ROOT
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(kw)
    return env


def _line(r):
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return lines[0]


def test_bench_one_rank_checks_every_element(gpu):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--slab-gib", "0.5", "--steps", "3",
                        "--warmup", "2", "--no-extra", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    line = _line(r)
    assert line["check_ok"] is True and "every element" in line["check"]
    assert line["n_gpus"] == 1 and line["roofline"]["kernel_ms_avg"] > 0


def test_c2_check_detects_a_wrong_element(gpu):
    """The C2 check is not vacuous: one flipped byte anywhere fails it."""
    import ctypes

    import torch

    sys.path.insert(0, ROOT)
    import bench
    from pnetcdf_amd import pncx

    lib = pncx.lib()
    sptr = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    wl = bench.C2Swap(torch, lib, sptr, 0.25, 1, 0)
    for _ in range(3):
        wl.launch()
    torch.cuda.synchronize()
    assert wl.check()
    wl._tbuf[wl._n - 5] ^= 1 << 40
    assert not wl.check()
    wl._tbuf[wl._n - 5] ^= 1 << 40
    wl.passes += 1                      # claims one pass too many: every element is now off
    assert not wl.check()
    wl.free()


def test_bench_two_ranks_gloo_twin(gpu):
    """The N > 1 path on one GPU: two ranks through bench.py's own launcher,
    gloo for the control plane, every rank's slab checked, the gather leg's
    checksums, and the rank report (shared device flagged)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--slab-gib", "0.25",
                        "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--gather-gib", "0.25",
                        "--gather-chunk-gib", "0.125", "--extra-steps", "3", "--extra-warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=_env(PNCX_DIST_BACKEND="gloo"), cwd=ROOT)
    line = _line(r)
    assert line["n_gpus"] == 2 and line["check_ok"] is True
    assert line["gather"]["checksums_ok"] is True and line["gather"]["chunks"] == 2
    # a gloo gather goes through the host: never reported as xGMI
    assert line["gather"]["via_xgmi"] is False
    # C3 and C4 per rank at N > 1, checks AND-reduced, kernel time per rank
    for name in ("c3", "c4", "c4_async", "c4_erange"):
        w = line["workloads"][name]
        assert w["check_ok"] is True and w["n_gpus"] == 2, name
        assert len(w["kernel_ms_per_rank"]) == 2 and w["value"] > 0, name
    assert "c1" not in line["workloads"]
    rk = line["ranks"]
    assert rk["world_size"] == 2 and rk["backend"] == "gloo" and rk["distinct_devices"] is False
    assert len(rk["kernel_ms_per_rank"]) == 2 and all(k > 0 for k in rk["kernel_ms_per_rank"])
