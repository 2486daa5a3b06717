"""Issue-cost estimate per basic block of one kernel in a hipcc -S file, from the measured per-instruction costs
(profiles/r04/isa_rates.txt, 4 waves per SIMD): 2.2 cycles for v_add/mul/fma_f32, v_add/sub_u32, v_and/or/xor_b32,
v_bitop3_b32, v_med3_f32 with VGPR operands only; 8 for f32 transcendentals; 16 for v_rcp_f64; 4 for every other
vector instruction (SGPR or literal operands included).  Scalar, memory and s_nop instructions are not counted.
  python3 scripts/isa_cost.py file.s <kernel substring>"""
import re
import sys

FAST = {"v_add_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_sub_f32", "v_subrev_f32", "v_add_u32", "v_sub_u32",
        "v_and_b32", "v_or_b32", "v_xor_b32", "v_bitop3_b32", "v_med3_f32", "v_mov_b32"}
TRANS = ("v_sqrt_f32", "v_rcp_f32", "v_exp_f32", "v_log_f32", "v_rsq_f32", "v_sin_f32", "v_cos_f32", "v_rcp_iflag_f32")


def cost(line):
    m = re.match(r"\s+(v_[a-z0-9_]+)\s*(.*)", line)
    if not m:
        return 0.0
    op, args = m.group(1), m.group(2)
    base = op.replace("_e32", "").replace("_e64", "")
    if base.startswith(TRANS):
        return 8.0
    if base == "v_rcp_f64" or base == "v_sqrt_f64":
        return 16.0
    if base in FAST and "dpp" not in op and not re.search(r"\bs\[?\d|0x|vcc|exec", args):
        return 2.2
    return 4.0


def main():
    s = open(sys.argv[1]).read()
    names = re.findall(r"^(_ZN5pfmpe\w+):", s, re.M)
    nm = [n for n in names if sys.argv[2] in n][0]
    i = s.index(nm + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j]
    parts = re.split(r"^(\.LBB\w+):(.*)$", body, flags=re.M)
    cur, note = "entry", ""
    rows = []
    for k in range(0, len(parts)):
        if k % 3 == 1:
            cur = parts[k]
            continue
        if k % 3 == 2:
            note = parts[k]
            continue
        lines = parts[k].splitlines()
        c = sum(cost(l) for l in lines)
        nv = sum(1 for l in lines if re.match(r"\s+v_", l))
        depth = note.count("Depth=") and re.findall(r"Depth=(\d)", note)
        rows.append((cur, nv, c, depth[-1] if depth else "0"))
    for r in rows:
        if r[1]:
            print(f"{r[0]:12s} valu {r[1]:4d} cost {r[2]:7.1f} depth {r[3]}")


if __name__ == "__main__":
    main()
