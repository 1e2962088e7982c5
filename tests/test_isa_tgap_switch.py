"""The round-4 tmode-7 aperture fault, examined on the ISA (CPU; VERDICT r04
"Next" 2).

Round 4 saw `HIP device error` from tests/test_gpu_flex.py::
test_flex_large_table while k_tgap chose the gap-map width at RUN time
(m.tmode == 6: 8-bit counts, a byte per element; else 4-bit steps scanned
across the wave) and blamed a miscompiled store address.  That kernel was
never committed; tools/isa/tgap_runtime_switch.hip reconstructs it beside
the shipped compile-time kernel, and this test compiles both for gfx950 (no
GPU) and reads them:

* The run-time kernel carries BOTH map reads into every launch: the 4-bit
  map's nibble loads (`toff8[q*32 + lane/2]`, inside the map) and the 8-bit
  map's per-element loads (`toff8[rc]`, rc up to tn - 1: past the end of a
  4-bit map, which holds tn/2 bytes).  Only an exec-mask branch keeps the
  second kind off a tmode-7 launch.  The shipped tmode-7 kernel has no
  per-element map load at all: 4 byte loads (one per unit in flight)
  against 8.
* The store addresses: every asm store's address is the 64-bit
  `c*tn + rc` of its unit, built by one v_mad_u64_u32 from a register pair
  whose high half is the zero register.  No "stale register" reaches a
  store in either kernel with this compiler.

So the reconstruction does not reproduce the round-4 claim; what the shipped
kernel removes structurally is the out-of-bounds-capable map read.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "isa", "tgap_runtime_switch.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc missing")
    out = tmp_path_factory.mktemp("isa") / "tgap.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-I", os.path.join(ROOT, "pnetcdf_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    SRC, "-o", str(out)], check=True, capture_output=True, timeout=600)
    s = out.read_text()
    kern = {}
    for name in re.findall(r"^(_Z\S+):", s, re.M):
        body = s[s.index(name + ":"):]
        kern["rt" if "k_tgap_rt" in name else "shipped"] = body[:body.find(".Lfunc_end")]
    assert set(kern) == {"rt", "shipped"}
    return kern


def test_runtime_switch_carries_the_per_element_map_load(isa):
    loads = {k: len(re.findall(r"global_load_ubyte", v)) for k, v in isa.items()}
    assert loads["shipped"] == 4, loads          # IMAP_U nibble loads, nothing per element
    assert loads["rt"] == 8, loads               # + the 8-bit map's toff8[rc] in every launch
    # both scan the nibbles across the wave (6 DPP adds per unit in flight)
    assert all(len(re.findall(r"_dpp ", v)) == 24 for v in isa.values())


def _store_address_sources(body):
    """For each asm store: the register pair fed to the v_mad_u64_u32 that
    builds its address, and whether that pair's high half was last written
    from the kernel's zero register."""
    lines = body.splitlines()
    zero = set()
    for ln in lines:                               # v_mov_b32 vN, 0 before the loop
        m = re.match(r"\s*v_mov_b32_e32 v(\d+), 0\s*$", ln)
        if m:
            zero.add(int(m.group(1)))
    out = []
    for k, ln in enumerate(lines):
        m = re.match(r"\s*global_store_dword v\[(\d+):(\d+)\], v\d+, off nt sc1", ln)
        if not m:
            continue
        a = int(m.group(1))
        mad = None
        for j in range(k - 1, max(0, k - 40), -1):
            mm = re.match(r"\s*v_mad_u64_u32 v\[%d:%d\], s\[\d+:\d+\], s\d+, v\d+, v\[(\d+):(\d+)\]" % (a, a + 1),
                          lines[j])
            if mm:
                mad = (int(mm.group(1)), int(mm.group(2)), j)
                break
        assert mad is not None, ln
        hi = mad[1]
        writer = None
        for j in range(mad[2] - 1, -1, -1):
            if re.match(r"\s*v_\S+ v%d\b|\s*v_\S+ v\[%d:" % (hi, hi), lines[j]) or \
               re.match(r"\s*v_\S+ v\[%d:%d\]" % (hi - 1, hi), lines[j]):
                writer = lines[j].strip()
                break
        out.append((ln.strip(), writer))
    return out, zero


def test_store_addresses_come_from_zero_extended_indices(isa):
    for name, body in isa.items():
        srcs, zero = _store_address_sources(body)
        assert len(srcs) == 4, (name, srcs)
        for store, writer in srcs:
            m = re.match(r"v_mov_b32_e32 v\d+, v(\d+)$", writer or "")
            assert (m and int(m.group(1)) in zero) or re.match(r"v_mov_b32_e32 v\d+, 0$", writer or ""), \
                (name, store, writer)


# ------------------------------------------------------------------------
# Round 6: every live-lane entry to the run-time kernel's per-element map
# load requires tmode == 6 (VERDICT r05 "Next" 5).  The kernel arguments are
# (src, dst, nunits, nq, pncxk_imap m, ...): m starts at byte 24, and
# offsetof(pncxk_imap, tmode / toff8) are compiled from pncx_shim.h here.

def _imap_offsets(tmp_path):
    c = tmp_path / "off.c"
    c.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "pncx.h"\n#include "pncx_shim.h"\n'
                 'int main(void){printf("%zu %zu\\n", offsetof(pncxk_imap, tmode), offsetof(pncxk_imap, toff8));'
                 'return 0;}\n')
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "pnetcdf_amd", "csrc"),
                    str(c), "-o", str(exe)], check=True, capture_output=True)
    tmode, toff8 = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    return 24 + tmode, 24 + toff8


def _pair(r):
    m = re.match(r"s\[(\d+):(\d+)\]$", r)
    return (int(m.group(1)), int(m.group(2))) if m else None


class _Cfg:
    """Blocks, labels and branch edges of one kernel body."""

    def __init__(self, body):
        self.lines = body.splitlines()
        self.label_at = {}                                   # label -> line index
        for k, ln in enumerate(self.lines):
            m = re.match(r"(\.LBB\d+_\d+):", ln)
            if m:
                self.label_at[m.group(1)] = k
        self.branches = []                                   # (line, opcode, target)
        for k, ln in enumerate(self.lines):
            m = re.match(r"\s*(s_cbranch_\w+|s_branch)\s+(\.LBB\d+_\d+)", ln)
            if m:
                self.branches.append((k, m.group(1), m.group(2)))

    def block_label(self, k):
        """the label (or None for a %bb comment block) starting the block of line k"""
        for j in range(k, -1, -1):
            ln = self.lines[j]
            m = re.match(r"(\.LBB\d+_\d+):", ln)
            if m:
                return m.group(1), j
            if re.match(r"; %bb\.\d+:", ln):
                return None, j
        return None, 0

    def prev_instr(self, j):
        for i in range(j - 1, -1, -1):
            s = self.lines[i].strip()
            if s and not s.startswith(";") and not s.startswith(".") and not s.endswith(":"):
                return i, s
        return None, ""

    def last_def(self, reg_re, k):
        """line index of the last instruction before k whose destination matches reg_re, checked to reach k
        on every path: no branch from outside (def, k] lands inside it"""
        defs = [d for d, ln in enumerate(self.lines) if re.match(r"\s*[sv]_\S+\s+" + reg_re + r"\s*,", ln)
                and not re.match(r"\s*(s_cmp|s_bitcmp|\S*_store)", ln)]        # compares write SCC, stores nothing
        for d in range(k - 1, -1, -1):
            if d in defs:
                for (b, _, tgt) in self.branches:
                    t = self.label_at[tgt]
                    if d < t <= k and not (d < b <= k):
                        # a back edge (b > k) is harmless when d is the register's only definition: every
                        # path past d executed d; a forward branch from before d would skip it
                        assert b > k and len(defs) == 1, (self.lines[d], self.lines[k], self.lines[b])
                return d
        raise AssertionError(f"no def of {reg_re} before line {k}")


def _meaning(cfg, reg, k, tmode_off):
    """'ne6' / 'eq6' for a mask register holding (m.tmode != 6) / (== 6) at line k"""
    d = cfg.last_def(re.escape(reg), k)
    ln = cfg.lines[d].strip()
    m = re.match(r"s_cselect_b64 (s\[\d+:\d+\]), -1, 0$", ln)
    if m:
        _, prev = cfg.prev_instr(d)
        mc = re.match(r"s_cmp_lg_u32 (s\d+), 6$", prev)
        assert mc, prev
        ld = cfg.last_def(re.escape(mc.group(1)), d)
        assert re.match(r"\s*s_load_dword %s, s\[0:1\], 0x%x$" % (re.escape(mc.group(1)), tmode_off), cfg.lines[ld]), \
            cfg.lines[ld]
        return "ne6"
    m = re.match(r"v_cmp_ne_u32_e64 (s\[\d+:\d+\]), 1, (v\d+)$", ln)
    if m:
        dv = cfg.last_def(re.escape(m.group(2)), d)
        mv = re.match(r"\s*v_cndmask_b32_e64 v\d+, 0, 1, (s\[\d+:\d+\])$", cfg.lines[dv])
        assert mv, cfg.lines[dv]
        return {"ne6": "eq6", "eq6": "ne6"}[_meaning(cfg, mv.group(1), dv, tmode_off)]
    raise AssertionError(f"unrecognised mask definition: {ln}")


def _jump_condition(cfg, k, tmode_off):
    """the tmode condition under which the vcc branch at line k is taken"""
    op = re.match(r"\s*(s_cbranch_vccz|s_cbranch_vccnz)\b", cfg.lines[k]).group(1)
    d = cfg.last_def("vcc", k)
    m = re.match(r"\s*(s_and_b64|s_andn2_b64) vcc, exec, (s\[\d+:\d+\])$", cfg.lines[d])
    assert m, cfg.lines[d]
    mean = _meaning(cfg, m.group(2), d, tmode_off)
    negate = (m.group(1) == "s_andn2_b64") != (op == "s_cbranch_vccz")
    return {"ne6": "eq6", "eq6": "ne6"}[mean] if negate else mean


def test_per_element_map_load_runs_only_under_tmode6(isa, tmp_path):
    """The run-time kernel's per-element map loads (toff8 + rc, rc up to
    tn - 1: 131,055 bytes past the 4-bit map of test_flex_large_table,
    tn = 262160, whose map holds 32 * 4097 bytes) sit in four blocks.  Each
    is entered either by `s_cbranch_execz` (no live lane: the load is
    inert) or by falling through from a block that only the tmode branch
    enters, and that branch is taken exactly when m.tmode == 6 (its mask
    traced to `s_cmp_lg_u32 <tmode>, 6` on the kernel-argument word of
    m.tmode).  So on a tmode-7 launch no live lane issues it; the shipped
    kernel has no such load at all."""
    tmode_off, toff8_off = _imap_offsets(tmp_path)
    for name, body in isa.items():
        cfg = _Cfg(body)
        toff8 = None
        for ln in cfg.lines:
            m = re.match(r"\s*s_load_dwordx(\d+) s\[(\d+):(\d+)\], s\[0:1\], 0x([0-9a-f]+)$", ln)
            if m and int(m.group(4), 16) <= toff8_off < int(m.group(4), 16) + 4 * int(m.group(1)):
                first = int(m.group(2)) + (toff8_off - int(m.group(4), 16)) // 4
                toff8 = f"s[{first}:{first + 1}]"
        assert toff8, name
        per_elem = []
        for k, ln in enumerate(cfg.lines):
            m = re.match(r"\s*global_load_ubyte v\d+, (v\[\d+:\d+\]), off$", ln)
            if not m:
                continue
            d = cfg.last_def(re.escape(m.group(1)), k)
            if re.match(r"\s*v_lshl_add_u64 %s, %s, 0, v\[\d+:\d+\]$" % (re.escape(m.group(1)), re.escape(toff8)),
                        cfg.lines[d]):
                per_elem.append(k)
        assert len(per_elem) == (4 if name == "rt" else 0), (name, per_elem)
        for k in per_elem:
            lab, start = cfg.block_label(k)
            assert lab is not None
            entries = [(b, op) for (b, op, t) in cfg.branches if t == lab]
            assert entries and all(op == "s_cbranch_execz" for _, op in entries), (lab, entries)
            # the fall-through predecessor: a block entered only by the tmode branch
            pi, prev = cfg.prev_instr(start)
            assert not prev.startswith("s_branch") and not prev.startswith("s_cbranch"), prev
            plab, pstart = cfg.block_label(pi)
            assert plab is not None
            into = [(b, op) for (b, op, t) in cfg.branches if t == plab]
            assert len(into) == 1 and into[0][1] in ("s_cbranch_vccz", "s_cbranch_vccnz"), (plab, into)
            _, before = cfg.prev_instr(pstart)
            assert before.startswith("s_branch"), before          # no fall-through into it
            assert _jump_condition(cfg, into[0][0], tmode_off) == "eq6", (lab, plab)
