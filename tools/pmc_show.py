"""Prints the last-dispatch value of every counter in gpurun_out/pmc*/ CSVs."""
import csv, glob, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(f"{root}/pmc*/**/*counter_collection.csv", recursive=True)):
    agg = {}
    for r in csv.DictReader(open(f)):
        agg.setdefault((r["Kernel_Name"][:40], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for (k, c), v in agg.items():
        print(f"{f.split('/')[1]:10s} {k:40s} {c:28s} {v[-1]:.6g}  (n={len(v)})")
