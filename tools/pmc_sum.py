"""Summarises one rocprofv3 --pmc pass (gpurun_out/<dir>/run_counter_collection.csv):
per-dispatch means of every counter, VALU busy (2 cycles per wave64
instruction per SIMD over GRBM_GUI_ACTIVE / 8 XCDs), VALU instructions per
16-byte block (--blocks N) and the wait fractions of wave time."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--blocks", type=float, default=2**30, help="16-byte blocks per dispatch")
ap.add_argument("--simds", type=int, default=1024)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
agg = collections.defaultdict(float)
disp = set()
for r in rows:
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    disp.add(r["Dispatch_Id"])
n = len(disp)
m = {k: v / n for k, v in agg.items()}
print(f"{n} dispatches, VGPR {rows[0]['VGPR_Count']} SGPR {rows[0]['SGPR_Count']} scratch {rows[0]['Scratch_Size']}")
for k, v in sorted(m.items()):
    print(f"  {k:24s} {v:.4g}")
if "GRBM_GUI_ACTIVE" in m:
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    if "SQ_INSTS_VALU" in m:
        print(f"  VALU busy {m['SQ_INSTS_VALU'] * 2 / (a.simds * cyc):.3f}, "
              f"VALU/block {m['SQ_INSTS_VALU'] * 64 / a.blocks:.1f}")
    if "SQ_INSTS_SALU" in m:
        print(f"  SALU/block {m['SQ_INSTS_SALU'] * 64 / a.blocks:.1f}")
if "SQ_WAVE_CYCLES" in m:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if k in m:
            print(f"  {k}/wave cycles {m[k] / m['SQ_WAVE_CYCLES']:.3f}")
