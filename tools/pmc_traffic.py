#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/profile.sh into
profiles/traffic.json: per config, the bulk kernel's HBM bytes per launch and
its LDS / VALU busy fractions, plus the FETCH/WRITE calibration copies.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half
of the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled
(`hbm_bytes_per_launch`, the guide's rule); WRITE_SIZE is exact for 16 B/lane
streaming stores.  Other access patterns are uncalibrated in the guide, so
tools/micro/calib_copy.hip copies a known byte count with each record access
pattern of the kernels and the ratio counted/known per pattern is stored under
"calibration" (DESIGN.md 5.1 reads the kernels' counts through it).

Usage: tools/pmc_traffic.py gpurun_out/r02 [profiles/traffic.json]
"""
import collections
import csv
import json
import os
import re
import sys

CALIB_PATTERNS = ("copy_stream", "copy_chacha", "copy_quad", "copy_gcm", "copy_gcm8",
                  "copy_quad_slow", "copy_quad_slow_t")
# Record geometry of each config's bench layout (length x stride): the
# counters' ratio to the bytes moved depends on it, so every config reads the
# calibration copy of its own geometry (calib_{fetch,write}_LENxSTRIDExRECS).
CONFIG_GEO = {"config2": "16384x16384", "config5": "16384x16384", "configG": "1350x1408",
              "config3": "1350x1408", "config3x": "1350x1408"}


def geo_known(geo, pattern):
    n_len, n_stride, n_recs = (int(x) for x in geo.split("x"))
    if pattern == "copy_stream":
        return n_recs * n_stride, n_recs * n_stride
    return n_recs * n_len, n_recs * (n_len + CALIB_TAGS_PER_REC)


def calib_pattern(full_name):
    """The calib_copy pattern of a bulk kernel instantiation's record reads:
    lanes per record L -> runs of 16 L bytes (gcm_kernel's last template
    argument; the keyset kernel and gcm_bs_kernel<..., 16> 16 lanes; ChaCha its
    own 64-byte-block pattern)."""
    if "chacha" in full_name:
        return "copy_chacha"
    m = re.search(r"gcm(?:_bs)?_kernel<([^>]*)>", full_name)
    lanes = int(m.group(1).split(",")[-1]) if m else 16
    if "keyset" in full_name:
        lanes = 16
    # (4 lanes: 64-byte runs, half a 128-byte line per record and iteration;
    # the kernel requests the two halves an iteration apart, and the counter
    # counts such requests near full size (0.95) where the back-to-back copy
    # counts half (0.55): the paced copy is the kernel's stream, round 6; the
    # T-table kernel's 4-lane loads are temporal since late round 6, the
    # table-free kernel's non-temporal)
    if lanes == 4 and "gcm_bs" not in full_name:
        return "copy_quad_slow_t"
    return {4: "copy_quad_slow", 8: "copy_gcm8", 16: "copy_gcm"}.get(lanes, "copy_gcm")
CALIB_TAGS_PER_REC = 16  # the copy kernels also write one 16-byte tag per record


def short_name(name):
    m = re.search(r"::(\w+)(<[^>]*>)?\(", name)  # bssl_amd::(anon)::gcm_kernel<...>(
    return m.group(1) if m else name.split("(")[0].split()[-1]  # copy_rec4<0>


def load(path):
    # Keyed by (kernel family, instantiation): a step may launch several
    # instantiations of one family (config 4: the long records at 8 lanes, the
    # short ones at 4), each once per step.
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    p = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(p):
        return out
    for r in csv.DictReader(open(p)):
        full = r["Kernel_Name"].split("(bssl_amd")[0]
        out[(short_name(r["Kernel_Name"]), full)][r["Counter_Name"]].append(
            float(r["Counter_Value"]))
    return out


def combine(entries):
    """One family's per-step figures from its instantiations' summaries: bytes
    summed (each runs once per step), busy and wait fractions weighted by each
    instantiation's cycles."""
    if len(entries) == 1:
        return entries[0]
    e = {"instantiations": len(entries)}
    for k in ("fetch_bytes_corrected", "write_bytes", "hbm_bytes_per_launch",
              "fetch_bytes_calibrated", "hbm_bytes_calibrated", "grbm_gui_active_per_xcd"):
        if all(k in x for x in entries):
            e[k] = sum(x[k] for x in entries)
    cyc = [x.get("grbm_gui_active_per_xcd", 0) for x in entries]
    for k in ("lds_busy", "valu_busy", "sq_wait_any_frac", "sq_wait_inst_any_frac"):
        if all(k in x for x in entries) and sum(cyc):
            e[k] = sum(x[k] * c for x, c in zip(entries, cyc)) / sum(cyc)
    return e


def summarise(c, full_name="", calib=None):
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    e = {"counters_avg_per_dispatch": avg}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = 2 * avg["FETCH_SIZE"] * 1024
        write = avg["WRITE_SIZE"] * 1024
        e.update({"fetch_bytes_corrected": fetch, "write_bytes": write,
                  "hbm_bytes_per_launch": fetch + write})
        # Calibrated: the counted bytes scaled by known / counted of the copy
        # kernel with the same record access pattern (tools/micro/calib_copy).
        pat = calib_pattern(full_name)
        cal = (calib or {}).get(pat, {})
        if cal.get("fetch_counted_over_known") and cal.get("write_counted_over_known"):
            fc = avg["FETCH_SIZE"] * 1024 / cal["fetch_counted_over_known"]
            wc = write / cal["write_counted_over_known"]
            e.update({"calib_pattern": pat, "fetch_bytes_calibrated": fc,
                      "hbm_bytes_calibrated": fc + wc})
    if "GRBM_GUI_ACTIVE" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / 8  # kernel cycles (GRBM sums the 8 XCDs)
        e["grbm_gui_active_per_xcd"] = cyc
        # Busy fractions of the units that can bind an integer kernel
        # (SQ_LDS_IDX_ACTIVE = LDS-array cycles summed over the 256 CUs; a
        # wave64 VALU instruction occupies its SIMD32 for >= 2 cycles, 1024 SIMDs).
        if "SQ_LDS_IDX_ACTIVE" in avg:
            e["lds_busy"] = avg["SQ_LDS_IDX_ACTIVE"] / 256 / cyc
        if "SQ_INSTS_VALU" in avg:
            e["valu_busy"] = avg["SQ_INSTS_VALU"] * 2 / 1024 / cyc
        if "SQ_WAVE_CYCLES" in avg:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if k in avg:
                    e[k.lower() + "_frac"] = avg[k] / avg["SQ_WAVE_CYCLES"]
    return e


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r02"
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    res = {}
    if os.path.exists(dst):  # merge: configs not profiled in `src` keep their entries
        res = json.load(open(dst))
    calib = collections.defaultdict(lambda: collections.defaultdict(dict))
    for sub in sorted(os.listdir(src)):
        m = re.match(r"calib_(fetch|write)_(\d+x\d+x\d+)$", sub)
        if not m:
            continue
        key = "FETCH_SIZE" if m.group(1) == "fetch" else "WRITE_SIZE"
        geo = m.group(2)
        for (k, _), c in load(os.path.join(src, sub)).items():
            name = {"copy_rec4<0>": "copy_chacha", "copy_rec4<1>": "copy_quad",
                    "copy_rec4<2>": "copy_quad_slow", "copy_rec4<3>": "copy_quad_slow_t",
                    "copy_gcm<16>": "copy_gcm", "copy_gcm<8>": "copy_gcm8"}.get(k, k.split("<")[0])
            if name not in CALIB_PATTERNS or key not in c:
                continue
            counted = sum(c[key]) / len(c[key]) * 1024
            known_r, known_w = geo_known(geo, name)
            if key == "FETCH_SIZE":
                calib[geo][name]["fetch_counted_over_known"] = counted / known_r
                calib[geo][name]["fetch_x2_over_known"] = 2 * counted / known_r
            else:
                calib[geo][name]["write_counted_over_known"] = counted / known_w
    if calib:
        res["calibration"] = {g: dict(v) for g, v in calib.items()}
        res["calibration_source"] = src
    calib_now = res.get("calibration", {})
    per_cfg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    for sub in sorted(os.listdir(src)):
        m = re.match(r"(?:bs_)?pmc_(config\w+?)_(fetch|write|sq)$", sub)
        if not m:
            continue
        for k, c in load(os.path.join(src, sub)).items():
            for n, v in c.items():
                per_cfg[m.group(1)][k][n].extend(v)
    for cfg, kernels in per_cfg.items():
        fam = collections.defaultdict(list)
        for (family, full), c in sorted(kernels.items()):
            geo = CONFIG_GEO.get(cfg)
            if cfg == "config4":  # mixed lengths: the long records at L = 8, the short at 4
                geo = "1350x1408" if calib_pattern(full) == "copy_quad" else "16384x16384"
            cal = next((v for g, v in calib_now.items() if geo and g.startswith(geo + "x")), None)
            fam[family].append(summarise(c, full, cal))
        # Merge by kernel family: a pass over one engine (ENGINE=bs runs of
        # tools/profile.sh) keeps the other engine's entries of the config.
        cur = res.get(cfg, {}) if isinstance(res.get(cfg), dict) else {}
        old_src = cur.pop("source", None)
        for k in cur:
            if isinstance(cur[k], dict) and old_src:
                cur[k].setdefault("source", old_src)
        for k, v in fam.items():
            cur[k] = combine(v)
            cur[k]["source"] = src
        res[cfg] = cur
    json.dump(res, open(dst, "w"), indent=1, sort_keys=True)
    for cfg, ks in res.items():
        if not isinstance(ks, dict):
            continue
        for k, e in ks.items():
            if not isinstance(e, dict):
                continue
            print(cfg, k, {x: (round(y / 1e9, 3) if isinstance(y, float) and y > 1e6 else
                               round(y, 3) if isinstance(y, float) else y)
                           for x, y in e.items() if x != "counters_avg_per_dispatch"})


if __name__ == "__main__":
    main()
