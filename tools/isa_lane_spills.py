"""Where a kernel's SGPR spills (v_writelane / v_readlane) and VGPR spills
(scratch) sit: per innermost loop of an hipcc -S listing, and in total.
usage: python tools/isa_lane_spills.py listing.s <kernel-name-substring> [max-loop-lines]"""
import re
import sys


def main():
    lines = open(sys.argv[1]).read().split('\n')
    key = sys.argv[2]
    span = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    start = next(n for n, l in enumerate(lines) if re.match(r'^_Z\S*:', l) and key in l.split(':')[0])
    end = start
    while not lines[end].strip().startswith('s_endpgm'):
        end += 1
    body = lines[start:end + 1]
    labels = {m.group(1): n for n, l in enumerate(body) if (m := re.match(r'^(\.LBB\d+_\d+):', l))}
    loops = []
    for n, l in enumerate(body):
        m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
        if m and labels.get(m.group(1), 1 << 30) < n and n - labels[m.group(1)] < span:
            loops.append((labels[m.group(1)], n))
    lane = [n for n, l in enumerate(body) if 'v_readlane' in l or 'v_writelane' in l]
    scr = [n for n, l in enumerate(body) if 'scratch_' in l]
    print(f"{key}: {len(body)} lines, lane spill ops {len(lane)}, scratch ops {len(scr)}, loops <= {span} lines: {len(loops)}")
    for a, b in loops:
        nl, ns = sum(a <= n <= b for n in lane), sum(a <= n <= b for n in scr)
        valu = sum(body[n].strip().startswith('v_') for n in range(a, b + 1))
        if nl or ns:
            print(f"  loop [{a}-{b}] valu {valu}: lane ops {nl}, scratch ops {ns}")


if __name__ == "__main__":
    main()
