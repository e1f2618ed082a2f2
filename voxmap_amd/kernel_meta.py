"""Per-kernel resource metadata of a built library (scratch, registers, spills).

Reads the gfx950 code object out of the library's ``.hip_fatbin`` section
(``llvm-objcopy`` + ``clang-offload-bundler``) and parses its AMDHSA metadata
note (``llvm-readelf --notes``).  ``check()`` is the guard ``build()`` runs:
the render kernels must keep 8 waves/SIMD (<= 64 VGPRs) and must not carry a
KernelArgs-sized private segment -- a pointer phi into the kernel arguments
makes the compiler copy the whole 1.7 KB struct to scratch per thread, which
fails silently (correct frames, ~14 GB of scratch traffic per frame).
DESIGN.md §3 lists the measured budgets.
"""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FIELDS = ("private_segment_fixed_size", "vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "group_segment_fixed_size")
RENDER_SCRATCH_LIMIT = 256      # bytes per thread: spill slots yes, a KernelArgs copy (~1.7 KB) no
STATS_SCRATCH_LIMIT = 512       # the counting (STATS) instantiations keep ~16 counters live: more spill slots
# VGPR spill slots allowed per EXT mode of a timed (non-STATS) k_render
# instantiation (0 v1, 1 extensions, 2 soft shadows, 3 pooled, 4 LDS bricks, 5/6
# general).  The rare paths (glass in draw order where panes stack, the stacked
# chain) spill at the 8-wave budget; what must never spill is a
# hot loop -- hot_loop_spills() checks the march and primary loops themselves.
# Each limit is the largest count of the current build plus a small margin
# (round 6, ADVICE r05: EXT 0 17, EXT 1 58, EXT 2 60, EXT 3 65, EXT 4 115,
# EXT 5 13, EXT 6 14 slots, all in tiled instantiations): a change that moves
# one is a change to look at, and the limit moves with it, measured.
# round 6: the sun march with the doom rule (its codes resolved after the
# step loop) reloads a few SGPR / scratch values inside the hard units' step
# loop; measured faster than the spill-free in-loop form on C3, v1 and
# REFLECT_ALL (profiles/r06_ab_doom10_c3.txt), so a handful is allowed there
HOT_LOOP_SPILL_LIMITS = {1: 8, 2: 2, 5: 8}
SPILL_LIMITS = {0: 19, 1: 62, 2: 64, 3: 70, 4: 132, 5: 16, 6: 16}
V1_SCRATCH_LIMIT = 72           # EXT 0's private segment (64 B now): the chain's slots, no KernelArgs copy
RENDER_VGPR_LIMIT = 64          # 8 waves/SIMD
GENERAL_VGPR_LIMIT = 96         # EXT 5/6: 5 waves/SIMD (their own unit, vx_render_e56.hip)


def _tool(name: str) -> str:
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else name


def code_objects(lib: str, d: str) -> list[str]:
    """The gfx950 code objects of ``lib``, unbundled into directory ``d``: the
    linker concatenates one offload bundle per HIP translation unit into the
    library's .hip_fatbin section."""
    fb = os.path.join(d, "fb.bin")
    subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                   check=True, capture_output=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for i, s in enumerate(starts):
        part, co = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"co{i}.o")
        with open(part, "wb") as f:
            f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--targets={TARGET}",
                        f"--input={part}", f"--output={co}"], check=True, capture_output=True)
        out.append(co)
    return out


def kernels(lib: str) -> dict[str, dict[str, int]]:
    """{mangled kernel name: {field: value}} for every kernel in ``lib``."""
    notes = ""
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(lib, d):
            notes += subprocess.run([_tool("llvm-readelf"), "--notes", co], check=True, capture_output=True,
                                    text=True).stdout
    # one YAML list item per kernel ("- .agpr_count: ..."), keys in alphabetical
    # order, so .group_segment_fixed_size precedes .name within the item
    out: dict[str, dict[str, int]] = {}
    blocks, cur = [], None
    for line in notes.splitlines():
        if re.match(r"\s+- \.", line):
            cur = {}
            blocks.append(cur)
        if cur is None:
            continue
        m = re.match(r"\s+(?:- )?\.name:\s+(\S+)$", line)
        if m:
            cur["__name"] = m.group(1)
            continue
        m = re.match(r"\s+(?:- )?\.(\w+):\s+(\d+)$", line)
        if m and m.group(1) in FIELDS:
            cur[m.group(1)] = int(m.group(2))
    for b in blocks:
        name = b.pop("__name", None)
        if name and "private_segment_fixed_size" in b:
            out[name] = b
    return out


def render_params(name: str):
    """(FMT, STATS, TILED, EXT, F32IDX) of a mangled k_render instantiation, else None."""
    m = re.search(r"k_render(?:_gen)?ILi(\d)ELb(\d)ELb(\d)ELi(\d)ELb(\d)E", name)
    return tuple(int(g) for g in m.groups()) if m else None


def hot_loop_spills(lib: str, ext_max: int = 6) -> dict[tuple, tuple[int, int]]:
    """(hot loops, spill instructions inside them) of each render kernel that
    renders frames (RGBA8, no stats, EXT <= ext_max).  Spill instructions: scratch_*,
    v_writelane, v_readlane.  Hot loops: the loops of the kernel's main body
    (before its first s_endpgm; the compiler places the rare paths after it)
    that are innermost, at most 400 instructions long, and hold a march texel
    load (buffer_load_format_x) or the primary walk's extent decode
    (v_cvt_f32_ubyte1): the step loops."""
    out: dict[tuple, tuple[int, int]] = {}
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(lib, d):
            txt = subprocess.run([_tool("llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            name, body = None, []
            for line in txt.splitlines() + ["0 <END>:"]:
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    p = render_params(name) if name else None
                    if p and p[0] == 1 and p[1] == 0 and p[3] <= ext_max:
                        out[p] = _hot_spills(body)
                    name, body = m.group(1), []
                elif name and "//" in line:
                    ins, cmt = line.split("//", 1)
                    am = re.match(r"\s*([0-9A-Fa-f]+):", cmt)
                    if am:
                        body.append((int(am.group(1), 16), ins.strip()))
    return out


def _hot_spills(body: list[tuple[int, str]]) -> tuple[int, int]:
    end = next((i for i, (_, l) in enumerate(body) if l.startswith("s_endpgm")), len(body))
    body = body[:end]
    index = {a: i for i, (a, _) in enumerate(body)}
    spill = [bool(re.match(r"(scratch_|v_writelane|v_readlane)", l)) for _, l in body]
    hot = [bool(re.match(r"(buffer_load_format_x\s|v_cvt_f32_ubyte1)", l)) for _, l in body]
    back = []                                             # backward branches: (loop head, latch)
    for i, (a, l) in enumerate(body):
        m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\d+)", l)
        if not m:
            continue
        off = int(m.group(1))
        off = off - 65536 if off >= 32768 else off        # simm16, printed unsigned
        tgt = index.get(a + 4 + 4 * off)                  # SOPP branch: PC + 4 + 4 * simm16
        if tgt is not None and tgt < i:
            back.append((tgt, i))
    loops = n = 0
    for h, e in back:                                     # innermost loops: the step loops themselves
        if (e - h > 400 or any(h <= h2 and e2 <= e and (h2, e2) != (h, e) for h2, e2 in back)
                or not any(hot[h:e + 1])):
            continue
        loops += 1
        n = max(n, sum(spill[h:e + 1]))
    return loops, n


def check(lib: str) -> dict[str, dict[str, int]]:
    """Raise if a render kernel copies its arguments to scratch or loses occupancy."""
    ks = kernels(lib)
    render = {k: v for k, v in ks.items() if "k_render" in k}
    if not render:
        raise RuntimeError(f"{lib}: no k_render kernels found in the gfx950 code object")
    bad = []
    for name, v in render.items():
        p = render_params(name)
        stats = p is not None and p[1] == 1                        # STATS instantiation: counting only
        # EXT 4 (VX_FLAG_SOFT_BRICK, an opt-in experiment): its 8 KB of LDS bricks
        # cap it at 7 waves/SIMD anyway, so the compiler may use 73 VGPRs
        brick = p is not None and p[3] == 4
        lim = STATS_SCRATCH_LIMIT if stats else RENDER_SCRATCH_LIMIT
        if v.get("private_segment_fixed_size", 0) > lim:
            bad.append(f"{name}: private segment {v['private_segment_fixed_size']} B > {lim}")
        # the timed product kernels: v1 and the extensions spill-free, soft shadows a
        # few VGPRs (scratch traffic in the hot path doubled the EXT 1 frame once)
        spill_lim = SPILL_LIMITS.get(p[3]) if p is not None and not stats else None
        if spill_lim is not None and v.get("vgpr_spill_count", 0) > spill_lim:
            bad.append(f"{name}: {v['vgpr_spill_count']} VGPRs spilled > {spill_lim}")
        # EXT 5/6 (glass in draw order, REFLECT_ALL): a budget of their own (vx_render_e56.hip, 5 waves/SIMD)
        general = p is not None and p[3] >= 5
        if not stats and v.get("vgpr_count", 0) > (80 if brick else GENERAL_VGPR_LIMIT if general else RENDER_VGPR_LIMIT):
            bad.append(f"{name}: {v['vgpr_count']} VGPRs > {RENDER_VGPR_LIMIT}")
    for p, (loops, n) in hot_loop_spills(lib).items():
        if not loops:
            bad.append(f"k_render{p}: no march / primary loop found in the disassembly (check the parser)")
        if n > HOT_LOOP_SPILL_LIMITS.get(p[3] if p else -1, 0):
            bad.append(f"k_render{p}: {n} spill instructions inside a march / primary loop")
    if bad:
        raise RuntimeError("render kernel resource check failed:\n  " + "\n  ".join(bad))
    return ks


if __name__ == "__main__":
    import sys
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "libvoxmap_hip.so")
    for name, v in sorted(kernels(lib).items()):
        print(f"{name[:70]:70s} " + " ".join(f"{f.split('_')[0][:5]}={v.get(f, 0)}" for f in FIELDS))
