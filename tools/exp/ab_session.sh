# Same-box A/B session (GPU box): for each "CFG:VARS" spec, REPS rounds of
# the current library (main) and each variant build (boringssl_amd/csrc/build/<v>),
# --no-parity (A/B timing only; parity is tested separately).
set -e
mkdir -p gpurun_out/ab; rm -f gpurun_out/ab/*.log
B=boringssl_amd/csrc/build
for spec in $SPECS; do
  CFG=${spec%%:*}; VARS=$(echo ${spec#*:} | tr ',' ' ')
  for rep in ${REPS:-1 2}; do
    timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/ab/${CFG}_main_$rep.log 2>&1
    for v in $VARS; do
      BSSL_AMD_LIB=$PWD/$B/$v/libbssl_amd.so timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/ab/${CFG}_${v}_$rep.log 2>&1
    done
  done
done
python3 - <<'PY'
import glob, json, os, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab/*.log")):
    name = os.path.basename(f)[:-4].rsplit("_", 1)[0]
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            res[name].append((d["value"], d["roofline"]["avg_kernel_ms"]))
for k, v in sorted(res.items()):
    print(f"{k:28s} " + "  ".join(f"{a:8.1f} GiB/s {b:8.3f} ms" for a, b in v))
PY
