#!/usr/bin/env python3
"""Where a kernel's scratch (spill) traffic sits: for each kernel symbol of a
hipcc device assembly file (hipcc --cuda-device-only -S), the compiler's
resource counts (.vgpr_spill_count / .private_segment_fixed_size) and every
scratch_load / scratch_store by the innermost natural loop that holds it
(a backward branch target .. branch), with the loop's size and its VALU /
LDS / vector-memory instruction counts, so the hot loops (the AES rounds, the
chunk and unit loops) can be told apart from the once-per-unit or
once-per-1,024-records code around them.

Usage: tools/isa_scratch.py build.s [kernel-name-regex] > report.txt
  (e.g. hipcc ... --cuda-device-only -S -DBSSL_BS_QUICK gcm_bs.hip -o bsq.s)
"""
import re
import subprocess
import sys


def demangle(name):
    try:
        out = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        return out.replace("bssl_amd::(anonymous namespace)::", "").split("(")[0]
    except OSError:
        return name


def kernels(lines):
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m and ".amdhsa_kernel " + m.group(1) in "".join(lines[i:i + 40000]):
            end = next(j for j in range(i + 1, len(lines)) if lines[j].startswith(".Lfunc_end"))
            yield m.group(1), i, end


def meta(lines, name):
    txt = "\n".join(lines)
    i = txt.find(".amdhsa_kernel " + name)
    blk = txt[i:i + 4000]
    g = lambda k: (re.search(k + r"\s+(\d+)", blk) or [None, "?"])[1]
    return {"private_segment_fixed_size": g(r"\.amdhsa_private_segment_fixed_size"),
            "next_free_vgpr": g(r"\.amdhsa_next_free_vgpr")}


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    lines = open(path).read().split("\n")
    for name, s, e in kernels(lines):
        dn = demangle(name)
        if pat and not pat.search(dn):
            continue
        labels = {}
        for i in range(s, e):
            m = re.match(r"^(\.LBB\d+_\d+):", lines[i])
            if m:
                labels[m.group(1)] = i
        loops = []
        for i in range(s, e):
            m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", lines[i])
            if m and m.group(1) in labels and labels[m.group(1)] < i:
                loops.append((labels[m.group(1)], i))
        def count(a, b, p):
            return sum(1 for l in lines[a:b + 1] if l.strip().startswith(p))
        print(f"== {dn}  {meta(lines, name)}  scratch ops: "
              f"{count(s, e, 'scratch_load')} loads, {count(s, e, 'scratch_store')} stores")
        rows = {}
        for i in range(s, e):
            st = lines[i].strip()
            if not st.startswith("scratch_"):
                continue
            inner = [lp for lp in loops if lp[0] <= i <= lp[1]]
            lp = min(inner, key=lambda x: x[1] - x[0]) if inner else None
            rows.setdefault(lp, []).append(st.split()[0])
        for lp, ops in sorted(rows.items(), key=lambda x: (x[0] or (0, 0))):
            if lp is None:
                print(f"   outside loops: {len(ops)} ({', '.join(sorted(set(ops)))})")
                continue
            a, b = lp
            print(f"   loop lines {a}-{b} ({b - a} lines: {count(a, b, 'v_')} VALU, "
                  f"{count(a, b, 'ds_')} LDS, {count(a, b, 'global_')} global): {len(ops)} scratch ops")
        hot = [lp for lp in loops if count(lp[0], lp[1], "v_bitop3") + count(lp[0], lp[1], "ds_read") > 500]
        for a, b in sorted(set(hot)):
            n = count(a, b, "scratch_")
            print(f"   hot loop {a}-{b}: {count(a, b, 'v_')} VALU, {count(a, b, 'ds_')} LDS, "
                  f"{n} scratch ops")


if __name__ == "__main__":
    main()
