cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in normal ablate1 ablate2; do
  if [ $v = normal ]; then L=""; else L="BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/$v/libbssl_amd.so"; fi
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/b_$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -o '"value": [0-9.]*\|"avg_kernel_ms": [0-9.]*' gpurun_out/b_$v.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
