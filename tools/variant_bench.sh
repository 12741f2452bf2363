#!/bin/bash
# Benchmarks diagnostic builds of the library (boringssl_amd/csrc/build/<v>/)
# against the default build, in one process per variant.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=""; else L="BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/$v/libbssl_amd.so"; fi
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} ${BENCH_ARGS:-} > gpurun_out/b_$v.log 2>&1; rc=$?
  echo "$v rc=$rc $(grep -o '"value": [0-9.]*\|"avg_kernel_ms": [0-9.]*' gpurun_out/b_$v.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
