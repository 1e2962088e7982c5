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


def _canned_full():
    """A whole bench result as worker() builds it: round 5's full line
    (profiles/r05zf_bench_default.json) with its C1 first-touch block in the
    interleaved form c1_first_touch now returns (2 runs per leg, phases)."""
    sys.path.insert(0, ROOT)
    import bench
    full = json.load(open(os.path.join(ROOT, "profiles", "r05zf_bench_default.json")))
    c1 = full["workloads"]["c1"]
    c1["legs"].pop("first_touch", None)
    order = bench.c1_first_order(2)
    phases = {f"put.{k}": [v, 1.0] for k, v in (("plan", 0.8), ("register", 1.9), ("convert", 18.2),
                                                  ("write", 487.8), ("grow", 244.1), ("total", 757.8))}
    runs = []
    for i, key in enumerate(order):
        if key == "ref":
            runs.append({"check_ok": True, "put_ms": 1.0 + 0.01 * i, "get_ms": 0.9, "put_ms_min": 0.9,
                         "get_ms_min": 0.85, "put_loop_ms": 40.0, "get_loop_ms": 29.0})
        else:
            runs.append({"put_ms": 0.8 + 0.01 * i, "get_ms": 0.3, "put_ms_min": 0.7, "get_ms_min": 0.25,
                         "put_loop_ms": 33.0, "get_loop_ms": 9.0, "close_ms": 0.02, "errors": 0,
                         "put_first_ms": 1.2, "get_first_ms": 0.9, "create_to_enddef_ms": 120.0,
                         "put_phases_us": {k.split(".")[1]: v[0] for k, v in phases.items()},
                         "put_phases": phases, "first_put_phases": phases, "get_phases": {"get.read": [174.9, 4.0]}})
    bench.c1_first_compare(order, runs)
    c1["first_touch"] = {"pattern": "x" * 200, "loops": "y" * 200, "order": order, "runs": runs, "check_ok": True}
    return bench, full


def test_bench_line_is_compact_and_keeps_every_workload():
    """The printed line stays under bench.LINE_MAX_CHARS (the driver keeps
    the tail of stdout; round 5's 10.8 KB line lost C3 and C4 from it) and
    still carries, per workload, its rate, roofline fraction and CPU
    baseline; C1 carries every interleaved run with its reference ratios."""
    bench, full = _canned_full()
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s) < bench.LINE_MAX_CHARS, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["roofline"]["frac"] > 0 and line["cpu_baseline"]["cores"] >= 1
    for name in ("c3", "c4", "c4_async", "c4_erange"):
        w = line["workloads"][name]
        assert w["roofline"]["frac"] > 0 and w["cpu_baseline"]["value"] > 0 and w["check_ok"], name
    ft = line["workloads"]["c1"]["first_touch"]
    assert ft["check_ok"] and ft["runs_in_order"].split()[0] == "ref"
    leg = ft["legs"]["host_8_io_threads"]
    assert len(leg["put_ms"]) == 2 and len(leg["put_vs_reference"]) == 2 and len(leg["put_loop_vs_reference"]) == 2
    assert leg["put_phases_us"]["write"] == 488
    assert len(ft["legs"]["reference_sequence"]["put_ms"]) == 3


def test_c1_first_order_interleaves_and_brackets():
    """Every library run has a reference run before and after it, every leg
    runs twice, and no leg is always the first after a reference run."""
    sys.path.insert(0, ROOT)
    import bench
    order = bench.c1_first_order(2)
    assert order[0] == "ref" and order[-1] == "ref"
    legs = [n for n, _, _ in bench.C1_LEGS]
    assert all(order.count(n) == 2 for n in legs)
    firsts = [order[i + 1] for i, k in enumerate(order[:-1]) if k == "ref"]
    assert len(set(firsts)) == 2
    runs = [{"check_ok": True, "put_ms": 1.0, "get_ms": 1.0, "put_loop_ms": 40.0} if k == "ref" else
            {"put_ms": 0.5, "get_ms": 0.25, "put_loop_ms": 20.0} for k in order]
    runs[0]["put_ms"] = 3.0                  # the first reference run only brackets the first round
    bench.c1_first_compare(order, runs)
    first_leg = runs[1]
    assert first_leg["put_vs_reference"] == 4.0      # (3.0 + 1.0) / 2 / 0.5
    assert runs[len(order) - 2]["put_vs_reference"] == 2.0
    assert all(r["get_vs_reference"] == 4.0 and r["put_loop_vs_reference"] == 2.0
               for k, r in zip(order, runs) if k != "ref")


def test_bench_line_compact_at_eight_ranks():
    """The N = 8 line (no C1; per-rank kernel times, the rank report and
    the gather leg added) also stays under the limit and keeps them."""
    bench, full = _canned_full()
    del full["workloads"]["c1"]
    full["n_gpus"] = 8
    for w in full["workloads"].values():
        w["kernel_ms_per_rank"] = [0.2512] * 8
        w["n_gpus"] = 8
    full["ranks"] = {"backend": "rccl", "world_size": 8, "local_device_of_rank0": "0000:05:00",
                     "distinct_devices": True, "pci_of_ranks": ["0000:%02x:00" % (5 + 16 * i) for i in range(8)],
                     "rccl_world_size": 8, "kernel_ms_per_rank": [10.0671] * 8}
    full["gather"] = {"collective": "gather into rank 0 (RCCL over xGMI)", "bytes_per_rank": 1 << 35,
                      "bytes_into_rank0": 7 << 35, "chunk_bytes_per_rank": 1 << 31, "chunks": 16, "ms": 400.0,
                      "GBps_into_rank0": 600.0, "checksums_ok": True, "via_xgmi": True, "pcie_ceiling_GBps": 57.5,
                      "note": "x" * 100}
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s) < bench.LINE_MAX_CHARS, len(s)
    assert line["ranks"]["distinct_devices"] and line["gather"]["checksums_ok"]
    assert all(len(w["kernel_ms_per_rank"]) == 8 for w in line["workloads"].values())
