#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_check.sh `pmc` step) into
profiles/traffic.json: HBM bytes per launch of each kernel.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half
of the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.
Usage: tools/pmc_traffic.py gpurun_out [profiles/traffic.json]
"""
import collections
import csv
import json
import os
import re
import sys


def load(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not sub.startswith("pmc") or not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            m = re.search(r"::(\w+)(<[^>]*>)?\(", name)
            short = m.group(1) if m else name
            out[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    data = load(src)
    res = {}
    for k, c in data.items():
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        e = {"counters_avg_per_dispatch": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            fetch = 2 * avg["FETCH_SIZE"] * 1024
            write = avg["WRITE_SIZE"] * 1024
            e.update({"fetch_bytes_corrected": fetch, "write_bytes": write,
                      "hbm_bytes_per_launch": fetch + write})
        if "GRBM_GUI_ACTIVE" in avg:
            cyc = avg["GRBM_GUI_ACTIVE"] / 8  # kernel cycles (GRBM sums the 8 XCDs)
            e["grbm_gui_active_per_xcd"] = cyc
            # Busy fractions of the compute units that can bind an integer
            # kernel (MI355X_MICROARCH.md: SQ_LDS_IDX_ACTIVE = LDS-array cycles,
            # summed over the 256 CUs; a wave64 VALU instruction occupies its
            # SIMD32 for 2 cycles, 1024 SIMDs).
            if "SQ_LDS_IDX_ACTIVE" in avg:
                e["lds_busy"] = avg["SQ_LDS_IDX_ACTIVE"] / 256 / cyc
            if "SQ_INSTS_VALU" in avg:
                e["valu_busy"] = avg["SQ_INSTS_VALU"] * 2 / 1024 / cyc
        res[k] = e
    json.dump(res, open(dst, "w"), indent=1, sort_keys=True)
    for k, e in res.items():
        print(k, {x: (round(y / 1e9, 3) if isinstance(y, float) else y) for x, y in e.items()
                  if x != "counters_avg_per_dispatch"})


if __name__ == "__main__":
    main()
