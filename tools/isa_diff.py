"""Which render kernels' machine code differs between two builds of the library.

Disassembles every gfx950 code object of both libraries (kernel_meta.code_objects),
cuts the listing per kernel, drops addresses and branch-target offsets, and
compares the instruction streams.  Used to check that a source change (a
translation-unit split, a new cold path) leaves the timed kernels' code as it was.

usage: python tools/isa_diff.py old.so new.so [substring filter]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from voxmap_amd import kernel_meta  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def listing(lib: str) -> dict[str, list[str]]:
    out: dict[str, list[str]] = {}
    with tempfile.TemporaryDirectory() as d:
        for co in kernel_meta.code_objects(lib, d):
            txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                                 text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    cur = out.setdefault(m.group(1), [])
                    continue
                if cur is None or not line.strip():
                    continue
                ins = line.split("//")[0].strip()
                ins = re.sub(r"<[^>]*>", "<L>", ins)              # branch targets
                if ins:
                    cur.append(ins)
    return out


def _norm(lines: list[str]) -> list[str]:
    # pc-relative constant addresses (s_getpc_b64 + s_add_u32/s_addc_u32 of an
    # offset to kPalette & co.) move with the code layout: compare them as offsets
    out = []
    for i, ins in enumerate(lines):
        if i >= 1 and lines[i - 1].startswith("s_getpc") and ins.startswith("s_add_u32"):
            ins = re.sub(r"0x[0-9a-f]+$", "<pcrel>", ins)
        out.append(ins)
    return out


def main():
    a, b = listing(sys.argv[1]), listing(sys.argv[2])
    filt = sys.argv[3] if len(sys.argv) > 3 else "k_render"
    same = diff = 0
    for name in sorted(set(a) | set(b)):
        if filt not in name:
            continue
        p = kernel_meta.render_params(name)
        la, lb = a.get(name), b.get(name)
        la, lb = la and _norm(la), lb and _norm(lb)
        if la == lb:
            same += 1
            continue
        diff += 1
        print(f"{p or name}: {len(la or [])} -> {len(lb or [])} instructions")
    print(f"identical {same}, different {diff}")


if __name__ == "__main__":
    main()
