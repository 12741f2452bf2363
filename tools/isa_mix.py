#!/usr/bin/env python3
"""Instruction mix of a kernel's hottest loop (hipcc --cuda-device-only -S
output): the innermost backward-branch loop with the most VALU instructions,
its instructions by issue class, and the VALU issue floor from the measured
per-wave-instruction costs at 4 waves per SIMD (tools/micro/valu_rate.hip,
profiles/r02/valu_rate.txt: add / xor / bitop3 / and / or / cndmask / mov
1.73-1.81 cycles ("fast"), alignbit / perm / alignbyte / lshl_or / add3 /
64-bit ops / multiplies 2.73-2.84 ("slow")).

Usage: tools/isa_mix.py file.s kernel-symbol-prefix [units-per-iteration]
"""
import collections
import re
import sys

FAST = 1.77
SLOW = 2.8
SLOW_OPS = ("v_alignbit", "v_alignbyte", "v_perm", "v_lshl_or", "v_add3", "v_mad_u64", "v_mad_i64",
            "v_mul_hi", "v_mul_lo", "v_mad_u32", "v_lshlrev_b64", "v_lshrrev_b64", "v_lshl_add_u64",
            "v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32", "v_mov_b64", "v_or3",
            "v_and_or", "v_xad", "v_lshl_add_u32", "v_add_lshl")


def classify(op):
    if op.startswith("v_"):
        return "valu_slow" if op.startswith(SLOW_OPS) else "valu_fast"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    units = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) and ":" in l)
    end = next(j for j in range(start + 1, len(lines)) if lines[j].startswith(".Lfunc_end"))
    labels = {}
    for i in range(start, end):
        m = re.match(r"^(\.LBB\d+_\d+):", lines[i])
        if m:
            labels[m.group(1)] = i
    loops = []
    for i in range(start, end):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)", lines[i])
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))

    def mix(a, b):
        c = collections.Counter()
        ops = collections.Counter()
        for l in lines[a:b + 1]:
            t = l.strip()
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            op = t.split()[0]
            c[classify(op)] += 1
            ops[op] += 1
        return c, ops

    best = max(loops, key=lambda lp: mix(*lp)[0]["valu_fast"] + mix(*lp)[0]["valu_slow"])
    c, ops = mix(*best)
    print(f"kernel {sym}\nhottest loop: lines {best[0]}-{best[1]} (per iteration; {units} units)")
    for k in ("valu_fast", "valu_slow", "lds", "vmem", "scratch", "salu", "waitcnt", "other"):
        print(f"  {k:10s} {c[k]:6d}  per unit {c[k] / units:8.1f}")
    cyc = FAST * c["valu_fast"] + SLOW * c["valu_slow"]
    print(f"  VALU issue floor at 4 waves/SIMD: {cyc:.0f} SIMD cycles per iteration "
          f"({cyc / units:.1f} per unit; {FAST} fast / {SLOW} slow)")
    print("  top opcodes: " + ", ".join(f"{o} {n}" for o, n in ops.most_common(14)))


if __name__ == "__main__":
    main()
