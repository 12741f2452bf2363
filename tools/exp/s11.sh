set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/al
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
for rep in 1 2; do
 for al in 128 16; do
  for v in main ab_l2; do
   if [ $v = main ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/$v/libbssl_amd.so; fi
   BSSL_AMD_ALIGN=$al timeout -k 10 300 python bench.py --config config3 --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/al/${v}_a${al}_$rep.log 2>&1 || exit 1
   echo "$v align=$al rep=$rep $(grep -o '"value": [0-9.]*' gpurun_out/al/${v}_a${al}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/al/${v}_a${al}_$rep.log)"
  done
 done
done
unset BSSL_AMD_LIB
