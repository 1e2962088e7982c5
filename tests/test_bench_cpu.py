"""bench.py's N-rank launcher (CPU): `--gpus N` without a torch.distributed
launcher starts N ranks itself, each seeing WORLD_SIZE=N; a WORLD_SIZE that
disagrees with --gpus is refused rather than reported as an N-GPU run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = ROOT
    return env


def test_launcher_sets_world_size():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--probe-launch"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["gpus_arg"] == 2 for x in lines)
    assert sorted(x["local_rank"] for x in lines) == [0, 1]


def test_launcher_refuses_mismatched_world():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--probe-launch"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 2 and "refusing" in r.stderr


def test_single_rank_needs_no_launcher():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--probe-launch"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line["world"] == 1 and line["rank"] == 0


def _c1_file(path, rec_offset, nbytes):
    with open(path, "wb") as f:
        f.write(b"\0" * (rec_offset + nbytes))


def test_c1_reference_sequences_move_the_right_bytes(tmp_path):
    """The C1 cpu_baseline restates the reference's calls (oracle/
    ref_sequence.c): put = swap in place, pwrite, swap back; get = malloc
    xbuf, pread, swap, memcpy into the user buffer, free.  Both functions
    compare every element read back with what was written (-2 otherwise);
    the first-touch form also appends each record past the end of the file
    and writes numrecs, whose big-endian bytes are checked here."""
    import ctypes
    import struct
    from oracle import oracle as O
    lib = O.lib()
    n, reps, off = 1 << 16, 3, 512
    p = tmp_path / "c1.nc"
    _c1_file(p, off, 4 * n)
    lib.orc_c1_sequence.restype = ctypes.c_int
    pm, gm = ctypes.c_double(0), (ctypes.c_double * 2)()
    assert lib.orc_c1_sequence(str(p).encode(), off, n, reps, ctypes.byref(pm), gm) == 0
    assert pm.value > 0 and gm[0] > 0 and gm[1] > 0
    raw = open(p, "rb").read()
    vals = struct.unpack(f">{n}I", raw[off:off + 4 * n])
    assert all(vals[i] == (i * 2654435761) & 0xffffffff for i in range(0, n, 997))
    # first touch: the file is cut back to its header, records appended
    nrec = 4
    lib.orc_c1_first_sequence.restype = ctypes.c_int
    o = (ctypes.c_double * 6)()
    assert lib.orc_c1_first_sequence(str(p).encode(), off, n, nrec, o) == 0
    raw = open(p, "rb").read()
    assert len(raw) == off + nrec * 4 * n
    assert struct.unpack(">Q", raw[4:12])[0] == nrec                 # numrecs (CDF-5)
    last = struct.unpack(f">{n}I", raw[off + (nrec - 1) * 4 * n:])
    assert all(last[i] == ((i * 2654435761) + nrec) & 0xffffffff for i in range(0, n, 997))
    assert all(x > 0 for x in o)
