#!/usr/bin/env python3
"""Steady-state kernel durations from a rocprofv3 --kernel-trace CSV
(`<dir>/run_kernel_trace.csv`): per kernel, the count, mean over every
dispatch (what `run_kernel_stats.csv` reports, cold calls included) and the
mean / median / min over the last N dispatches (the bench's timed steps:
`bench.py --steps N` runs its warm-up calls first).  The steady mean is the
figure to set beside a bench line's `ms_per_step`.

Usage: tools/kstats_steady.py DIR_OR_CSV [--last N] [--json OUT]"""
import argparse
import csv
import json
import os
import re
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("--last", type=int, default=10)
ap.add_argument("--json")
a = ap.parse_args()
path = a.src
if os.path.isdir(path):
    cands = [os.path.join(dp, f) for dp, _, fs in os.walk(path) for f in fs
             if f.endswith("kernel_trace.csv")]
    path = sorted(cands)[0]
rows = {}
for r in csv.DictReader(open(path)):
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(bssl_amd")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
    rows.setdefault(name, []).append((int(r["Start_Timestamp"]), d))
out = {}
for name, v in sorted(rows.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
    v.sort()
    ds = [x[1] for x in v]
    last = ds[-a.last:]
    out[name] = {"count": len(ds), "mean_all_us": round(statistics.mean(ds), 2),
                 "steady_last": len(last), "steady_mean_us": round(statistics.mean(last), 2),
                 "steady_median_us": round(statistics.median(last), 2),
                 "steady_min_us": round(min(last), 2), "max_us": round(max(ds), 2)}
    print(f"{len(ds):5d} all {out[name]['mean_all_us']:10.2f}  last{len(last)} mean "
          f"{out[name]['steady_mean_us']:10.2f} med {out[name]['steady_median_us']:10.2f}  {name[:100]}")
if a.json:
    json.dump({"source": path, "kernels": out}, open(a.json, "w"), indent=1)
