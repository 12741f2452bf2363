#!/usr/bin/env python3
"""Per-kernel register / spill / scratch table of one HIP source for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage).  Usage:
  python tools/kres.py boringssl_amd/csrc/gcm.hip [extra hipcc flags] [--filter SUBSTR]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
args = sys.argv[1:]
flt = None
if "--filter" in args:
    i = args.index("--filter")
    flt = args[i + 1]
    del args[i:i + 2]
src, extra = args[0], args[1:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
       f"-I{ROOT}/include", f"-I{ROOT}/boringssl_amd/csrc", "-fvisibility=hidden",
       "-munsafe-fp-atomics", "--cuda-device-only", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        name = re.sub(r"bssl_amd::\(anonymous namespace\)::", "", name)
        name = re.sub(r"\(.*", "", name)
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt and flt not in r["name"]:
        continue
    print(f"{r['name'][:70]:70s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} "
          f"vspill {r.get('VGPRs Spill', '?'):>4s} sspill {r.get('SGPRs Spill', '?'):>4s} "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4s} occ {r.get('Occupancy [waves/SIMD]', '?')}")
