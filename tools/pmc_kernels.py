#!/usr/bin/env python3
"""Per-kernel means of the counters in rocprofv3 --pmc CSV output
(`<dir>/**/*counter_collection.csv`): for each kernel, the number of
dispatches and the mean per dispatch of every counter collected, plus the
derived per-wave instruction counts.  Usage: tools/pmc_kernels.py DIR [...]"""
import collections
import csv
import os
import re
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(set)
    for dp, _, fs in os.walk(path):
        for f in fs:
            if not f.endswith("counter_collection.csv"):
                continue
            for r in csv.DictReader(open(os.path.join(dp, f))):
                name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(bssl_amd")[0]
                agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
                ndisp[name].add(r["Dispatch_Id"])
    return agg, ndisp


for path in sys.argv[1:]:
    agg, ndisp = load(path)
    print("==", path)
    for name, c in agg.items():
        n = len(ndisp[name])
        mean = {k: v / n for k, v in c.items()}
        waves = mean.get("SQ_WAVES", 0) or 1
        extra = ""
        if "SQ_INSTS_VALU" in mean:
            extra = (f" valu/wave {mean['SQ_INSTS_VALU'] / waves:.0f} lds/wave "
                     f"{mean.get('SQ_INSTS_LDS', 0) / waves:.0f} vmem/wave "
                     f"{mean.get('SQ_INSTS_VMEM', 0) / waves:.0f}")
            if mean.get("SQ_WAVE_CYCLES"):
                extra += (f" wait_any {mean.get('SQ_WAIT_ANY', 0) / mean['SQ_WAVE_CYCLES']:.3f}"
                          f" wait_inst {mean.get('SQ_WAIT_INST_ANY', 0) / mean['SQ_WAVE_CYCLES']:.3f}")
        print(f"  {n:3d} {name[:70]}{extra}")
        print("      " + " ".join(f"{k}={v:.4g}" for k, v in sorted(mean.items())))
