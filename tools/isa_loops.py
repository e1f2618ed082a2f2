"""Loops of one kernel in an hipcc -S listing: per backward branch, its VALU,
vector-memory and scratch instruction counts (which loop carries spills).
usage: python tools/isa_loops.py listing.s <kernel-name-substring>"""
import re
import sys


def kernel_body(lines, key):
    for i, l in enumerate(lines):
        if re.match(r'^_Z\S*:', l) and key in l.split(':')[0]:
            j = i
            while not lines[j].strip().startswith('s_endpgm'):
                j += 1
            return lines[i:j + 1]
    raise SystemExit(f"no kernel matching {key}")


def main():
    lines = open(sys.argv[1]).read().split('\n')
    body = kernel_body(lines, sys.argv[2])
    labels = {}
    for n, l in enumerate(body):
        m = re.match(r'^(\.LBB\d+_\d+):', l)
        if m:
            labels[m.group(1)] = n
    print(f"{len(body)} lines, scratch ops {sum('scratch_' in x for x in body)}")
    for n, l in enumerate(body):
        m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
        if m and labels.get(m.group(1), 1 << 30) < n:
            seg = body[labels[m.group(1)]:n + 1]
            cnt = lambda p: sum(1 for x in seg if re.match(p, x))
            valu, vmem, salu = cnt(r'\s+v_'), cnt(r'\s+(buffer|global)_load'), cnt(r'\s+s_')
            scr = sum('scratch_' in x for x in seg)
            print(f"loop {m.group(1)} [{labels[m.group(1)]}-{n}]: valu {valu}, vmem {vmem}, scratch {scr}, salu {salu}")


if __name__ == "__main__":
    main()
