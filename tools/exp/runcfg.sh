# Same-box A/B of library builds on a bench config: CFG, VARS (build dirs).
set -e
mkdir -p gpurun_out
B=boringssl_amd/csrc/build
for rep in ${REPS:-1 2}; do
  timeout -k 10 200 python bench.py --config $CFG --steps ${STEPS:-5} --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/c_${CFG}_main_$rep.log 2>&1
  for v in ${VARS:-}; do
    BSSL_AMD_LIB=$PWD/$B/$v/libbssl_amd.so timeout -k 10 200 python bench.py --config $CFG --steps ${STEPS:-5} --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/c_${CFG}_${v}_$rep.log 2>&1
  done
done
