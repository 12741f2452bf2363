#!/usr/bin/env python3
"""Per-kernel duration summary (count, mean, median, min, max in us) from a
rocprofv3 sqlite output (the default .db format): tools/kstats_db.py FILE.db"""
import sqlite3
import statistics
import sys

c = sqlite3.connect(sys.argv[1])
rows = {}
for name, d in c.execute("select name, duration from kernels"):
    rows.setdefault(name.replace("(anonymous namespace)::", "").split("(")[0][:90], []).append(d / 1000.0)
for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    print(f"{len(v):6d}  mean {statistics.mean(v):9.2f}  med {statistics.median(v):9.2f}  "
          f"min {min(v):9.2f}  max {max(v):9.2f}  {name}")
