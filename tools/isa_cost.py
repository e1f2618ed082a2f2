"""Static VALU-cycle pricing of a kernel's ISA with the gfx950 cost table of
profiles/r01_valu_costs.txt: per basic block, SIMD-cycles of VALU issue
(2 for add/mul/fma/logic/mov, 4 for floor/cvt/min3/med3/cmp/cndmask/u24/add3
and packed ops, 8 for transcendentals), SALU and memory instruction counts.
Usage: python tools/isa_cost.py kernel.s [top_n]"""
import re
import sys

FOUR = ("v_floor", "v_ceil", "v_trunc", "v_rndne", "v_fract", "v_cvt", "v_min3", "v_max3", "v_med3", "v_cmp", "v_cndmask",
        "v_mul_u32_u24", "v_mul_i32_i24", "v_mad_u32_u24", "v_mad_i32_i24", "v_add3", "v_pk_", "v_lshl_add", "v_add_lshl",
        "v_lshl_or", "v_and_or", "v_or3", "v_xad", "v_bfe", "v_bfi", "v_alignbit", "v_perm", "v_ldexp", "v_frexp",
        "v_div_fixup", "v_div_scale", "v_div_fmas", "v_mad_u64", "v_lshl_add_u64", "v_mul_hi", "v_mul_lo", "v_subrev_co",
        "v_sub_co", "v_add_co", "v_addc", "v_subb", "v_cmpx", "v_readfirstlane", "v_readlane", "v_writelane", "v_mbcnt")
EIGHT = ("v_sqrt", "v_rcp", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos")


def cost(op):
    if op.startswith(EIGHT):
        return 8
    if op.startswith(FOUR):
        return 4
    return 2


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    blocks, cur = [], None
    for line in open(path):
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?(.*)", line)
        if m:
            cur = {"name": m.group(1), "note": m.group(2).strip(), "valu": 0, "n_valu": 0, "salu": 0, "vmem": 0, "lds": 0}
            blocks.append(cur)
            continue
        t = line.strip().split()
        if not t or cur is None or t[0].startswith((";", ".")):
            continue
        op = t[0]
        if op.startswith("v_"):
            cur["valu"] += cost(op)
            cur["n_valu"] += 1
        elif op.startswith("s_"):
            cur["salu"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            cur["vmem"] += 1
        elif op.startswith("ds_"):
            cur["lds"] += 1
    tot = sum(b["valu"] for b in blocks)
    print(f"total static VALU cycles {tot} in {len(blocks)} blocks")
    for b in sorted(blocks, key=lambda b: -b["valu"])[:top]:
        print(f"{b['name']:14s} valu {b['valu']:5d} ({b['n_valu']:4d} instr) salu {b['salu']:3d} vmem {b['vmem']:2d} "
              f"lds {b['lds']:2d} {b['note'][:60]}")


if __name__ == "__main__":
    main()
