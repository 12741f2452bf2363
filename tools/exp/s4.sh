# config 3 write traffic: non-temporal vs plain ciphertext stores (PMC + timing)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
B="python3 bench.py --config config3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity"
for v in main ab_nts0; do
  if [ $v = main ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/$v/libbssl_amd.so; fi
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-include-regex chacha_poly_kernel --pmc $c -d gpurun_out/pmc/${v}_$c -o run --output-format csv -- $B > gpurun_out/pmc/${v}_$c.log 2>&1 || exit 1
  done
done
unset BSSL_AMD_LIB
SPECS="config3:ab_nts0" REPS="1 2" timeout -k 10 600 bash tools/exp/ab_session.sh > gpurun_out/ab_nts.txt 2>&1; cat gpurun_out/ab_nts.txt
python3 - <<'PY'
import csv,glob
for f in sorted(glob.glob("gpurun_out/pmc/*/**/*counter_collection.csv", recursive=True)):
    vals=[float(r["Counter_Value"]) for r in csv.DictReader(open(f))]
    print(f.split("/")[2], len(vals), sum(vals)/max(1,len(vals)))
PY
SPECS="config3:ab_abl2,ab_abl3,ab_abl7,ab_abl8" REPS="1 2" timeout -k 10 900 bash tools/exp/ab_session.sh > gpurun_out/ab_abl.txt 2>&1; cat gpurun_out/ab_abl.txt
