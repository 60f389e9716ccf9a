"""Device-assembly check of the fused kernels (CPU only: hipcc cross-compiles gfx950).

tools/mfma_lint.py follows every MFMA along all control-flow paths and flags inline-asm
instructions that (a) write a register of the MFMA's destination before anything has read it
(WAW: the MFMA's write-back can land after the asm result; round 2 hit this in layer 3), or
(b) write a register the MFMA reads as srcC within its pass window (WAR: a multi-pass MFMA reads
srcC late), (c) read the MFMA's result before its latency has passed, or (d) write a register a
following MFMA reads fewer than 2 wait states later.  The compiler's hazard checks do not cover
inline asm.  The build must show none of them.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
sys.path.insert(0, os.path.join(ROOT, "tools"))

import mfma_lint  # noqa: E402

SYNTHETIC = """\
_Z3fooPi:
	v_mov_b32_e32 v8, 0
.LBB0_1:
	v_mfma_i32_16x16x64_i8 v[0:3], v[4:7], v[12:15], v[8:11]
	v_add_u32_e32 v20, v0, v1
	s_cbranch_scc1 .LBB0_1
	;;#ASMSTART
	v_ashr_pk_i8_i32 v9, v20, v21, 0
	;;#ASMEND
	s_endpgm
_Z3barPi:
.LBB1_1:
	;;#ASMSTART
	v_ashr_pk_i8_i32 v10, v20, v21, 0
	;;#ASMEND
	s_nop 0
	v_mfma_i32_16x16x64_i8 v[0:3], v[4:7], v[12:15], v[8:11]
	s_nop 1
	s_branch .LBB1_1
_Z3bazPi:
	v_mfma_i32_16x16x64_i8 v[0:3], v[4:7], v[12:15], v[8:11]
	s_nop 4
	;;#ASMSTART
	v_ashr_pk_i8_i32 v9, v20, v21, 0
	;;#ASMEND
	v_mfma_i32_32x32x32_i8 v[32:47], v[4:7], v[12:15], 1.0
	s_cbranch_execz .LBB2_9
	v_add_u32_e32 v50, v1, v2
.LBB2_9:
	;;#ASMSTART
	v_ashr_pk_i8_i32 v40, v20, v21, 0
	;;#ASMEND
	s_endpgm
_Z3quxPi:
	v_mfma_i32_16x16x64_i8 v[0:3], v[4:7], v[12:15], v[8:11]
	s_nop 3
	;;#ASMSTART
	v_ashr_pk_i8_i32 v30, v0, v1, 0
	;;#ASMEND
	;;#ASMSTART
	v_ashr_pk_i8_i32 v13, v20, v21, 0
	;;#ASMEND
	v_mfma_i32_16x16x64_i8 v[40:43], v[4:7], v[12:15], 0
	s_endpgm
"""


def test_lint_finds_hazards_across_branches(tmp_path):
    p = tmp_path / "syn.s"
    p.write_text(SYNTHETIC)
    with open(os.devnull, "w") as null:
        found = mfma_lint.lint(str(p), out=null)
    whys = {}
    for (line, why) in found:
        whys.setdefault(line, []).append(why)
    has = lambda line, tag: any(tag in w for w in whys.get(line, []))  # noqa: E731
    assert has(8, "WAR")               # fall-through after a conditional branch
    assert has(14, "WAR")              # across a loop back edge (write at the loop head)
    assert has(14, "RAW, needs 2")     # ... which is also read 1 wait state later by the MFMA
    assert has(31, "pending dst")      # on the taken side of s_cbranch_execz
    assert 24 not in whys and 23 not in whys             # 5 wait states after a 4-pass MFMA: outside the WAR window
    assert has(38, "RAW, window 8")    # asm reads a 4-pass MFMA's result 4 states after it
    assert has(41, "RAW, needs 2")     # MFMA reads an asm output with no wait state between
    assert has(38, "asm first reader")  # ... and no compiler-emitted instruction read it first
    assert len(found) == 7


def test_no_inline_asm_hazard_next_to_mfma(device_asm):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_lint.py"), str(device_asm)],
                       check=True, capture_output=True, text=True)
    hazards = [l for l in r.stdout.splitlines() if "asm write into" in l or "asm first reader" in l]
    assert not hazards, "\n".join(hazards)


def test_lint_flags_the_round5_clamp_form():
    """Round 5's clamp-bit layer-2 form (a) returned wrong logits on the GPU at random; form (b),
    the same arithmetic with a compiler-emitted first reader of the accumulator, was exact
    (DESIGN.md §3).  The lint's asm-first-reader rule flags the failing build's device code (an
    excerpt committed as a fixture) on all eight accumulator pairs and nothing in form (b); the
    shipped build stays clean (test_no_inline_asm_hazard_next_to_mfma)."""
    golden = os.path.join(ROOT, "tests", "golden")
    with open(os.devnull, "w") as null:
        bad = mfma_lint.lint(os.path.join(golden, "r05_clamp_form_a.s"), out=null)
        good = mfma_lint.lint(os.path.join(golden, "r05_clamp_form_b.s"), out=null)
    first = sorted(line for (line, why) in bad if "asm first reader" in why)
    assert len(first) == 8, bad
    assert not good, good


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    """gfx950 assembly of the library's kernels (one compile per module)."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    asm = tmp_path_factory.mktemp("asm") / "mibminet.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function",
                    "-mllvm", "-disable-promote-alloca-to-lds", "--cuda-device-only", "-S", "-o", str(asm),
                    os.path.join(ROOT, "mi-bminet_amd", "csrc", "mibminet.hip")],
                   check=True, capture_output=True)
    return asm


def _functions(asm):
    import re
    funcs, name = {}, None
    for line in open(asm):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name = m.group(1)
            funcs[name] = []
        elif name:
            funcs[name].append(line.strip())
    return funcs


def test_trial_loop_barriers_do_not_drain_prefetch(device_asm):
    """Every k_forward keeps its next-trial loads in flight across the trial loop's barriers: no
    s_barrier but the one before the loop is preceded by an s_waitcnt on vmcnt.  The channel-major LDS-DMA
    fill is inline asm for this reason: with __builtin_amdgcn_raw_ptr_buffer_load_lds
    the compiler puts vmcnt(0) before every __syncthreads().  The DMA instructions set m0 themselves,
    and nothing else in these kernels touches m0.  (LDS-DMA serves the 22-channel shapes only: the
    channel-major int8 ring, and the blocks past the VGPR prefetch of time-major plain BN and exact
    division.)"""
    funcs = {n: ls for n, ls in _functions(device_asm).items() if "2wg9k_forward" in n}
    assert len(funcs) == 72
    n_dma = 0
    for name, lines in funcs.items():
        barriers = [i for i, l in enumerate(lines) if l.startswith("s_barrier")]
        assert len(barriers) >= 3, name
        for i in barriers[1:]:
            waits = [l for l in lines[max(0, i - 4):i] if l.startswith("s_waitcnt")]
            assert not waits or "vmcnt" not in waits[-1], (name, lines[i - 4:i + 1])  # the barrier's own wait
        code = [l.split(";")[0].strip() for l in lines]
        for i, l in enumerate(code):
            ops = l.replace(",", " ").split()
            if "m0" not in ops:
                continue
            # m0 only ever holds the LDS base of the next DMA load: written right before it (the
            # compiler writes it for the asm's "{m0}" operand), read by nothing else
            assert ops[1] == "m0" and ops[0].startswith("s_"), (name, l)
            nxt = next(c for c in code[i + 1:] if c and not c.startswith(".") and "m0" in c.replace(",", " ").split()
                       or c.endswith(" lds"))
            assert nxt.startswith("buffer_load_dwordx4") and nxt.endswith(" lds"), (name, l, nxt)
        dma = sum(1 for l in lines if l.startswith("buffer_load_dwordx4") and l.endswith(" lds"))
        assert (dma > 0) == (_dma_kind(name) is not None), (name, dma)
        n_dma += dma > 0
    assert n_dma == 14


def _dma_kind(name):
    """Cfg<C, T, RB, CB, CT, FQ, XR>: "ring" for channel-major int8 22-ch, "ldma" for time-major plain
    BN or exact-division 22-ch (int8 input), None for the rest."""
    c = _cfg(name)
    if c[0] != 22 or c[5]:
        return None
    return "ring" if c[4] else "ldma" if (not c[2] or c[6]) else None


def _cfg(name):
    import re
    m = re.search(r"CfgILi(\d+)ELi(\d+)((?:ELb[01])+)E", name)
    return tuple(int(v) for v in (m.group(1), m.group(2))) + tuple(int(b) for b in re.findall(r"Lb([01])", m.group(3)))


def test_dma_ring_wait_counts_issued_ops(device_asm):
    """Layer 1 of the LDS-DMA kernels waits for the fill with a fixed s_waitcnt vmcnt(N) (inline asm,
    forward_wg.hpp layer1).  Channel-major ring: N = 1 on the last wave, whose previous trial's
    logits store was issued after the fill and need not complete, 0 elsewhere.  Time-major plain BN
    and exact division: N = PF, the VGPR prefetch loads issued right after the LDS-DMA ones.  That is only safe while at
    least N vector-memory operations follow the trial loop's last fill.  Scratch
    traffic (spills) after the fill only makes the wait stricter."""
    import re
    funcs = {n: ls for n, ls in _functions(device_asm).items() if "2wg9k_forward" in n}
    checked = 0
    for name, lines in funcs.items():
        fills = [i for i, l in enumerate(lines) if l.startswith("buffer_load_dwordx4") and l.endswith(" lds")]
        if not fills:
            continue
        # the trial loop: the last depth-1 loop header before the last fill
        head = max(i for i, l in enumerate(lines[:fills[-1]]) if re.search(r"=>This (Inner )?Loop Header: Depth=1", l))
        loop_fills = [i for i in fills if i > head]
        assert loop_fills, name
        waits, in_asm = [], False
        for i, l in enumerate(lines):
            if l.startswith(";;#ASMSTART"):
                in_asm = True
            elif l.startswith(";;#ASMEND"):
                in_asm = False
            elif in_asm and i > head and l.startswith("s_waitcnt vmcnt("):
                waits.append(int(l.split("(")[1].split(")")[0]))
        kind = _dma_kind(name)
        # (vmcnt(0) after the loop: the last fill lands before the wave ends)
        assert sorted(set(waits)) == ([0, 1] if kind == "ring" else [0, 3]), (name, kind, waits)
        after = [l for l in lines[loop_fills[-1] + 1:]
                 if l.startswith(("global_store", "buffer_store", "global_load", "buffer_load")) and not l.endswith(" lds")]
        if kind == "ring":
            after = [l for l in after if l.startswith("global_store_dword ")]
        assert len(after) >= max(waits), (name, after)
        checked += 1
    assert checked == 14


def test_layer1_cinit_not_written_near_loads(device_asm):
    """The round-1 layer-1 fault's remaining candidate: an MFMA C-init written by a
    VALU instruction a few wait states before the MFMA while loads are outstanding.  In every
    k_forward instantiation (time-major, channel-major, float input; all build variants) the
    layer-1 C-inits are built once before the trial loop (where a full drain precedes the first
    layer 1), so no layer-1 MFMA may show the pattern (tools/cinit_scan.py)."""
    import cinit_scan

    asm = device_asm
    with open(os.devnull, "w") as null:
        old, sys.stdout = sys.stdout, null
        try:
            hits = cinit_scan.scan(cinit_scan.parse(str(asm)), [])
        finally:
            sys.stdout = old
    funcs = [n for n in cinit_scan.parse(str(asm)) if "2wg9k_forward" in n]
    assert len(funcs) == 72
    assert not [h for h in hits if h[1] == 1], [h for h in hits if h[1] == 1]
