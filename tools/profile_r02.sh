#!/bin/bash
# Round-2 profiling session (one GPU): counter list, config 2 read-traffic
# attribution (full build vs. the no-plaintext-load ablation), and rocprofv3
# stats + FETCH/WRITE/SQ passes for configs 4 and 5.  Output under
# gpurun_out/r02/.  Each GPU step has its own limit; the chain stops at the
# first failure other than a test failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r02
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  [ $rc -eq 0 ] || exit $rc
}
B2="python3 bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline --records 262144"
step counters 120 rocprofv3 -L
for v in full ablate3 ablate4; do
  lib=boringssl_amd/libbssl_amd.so
  [ $v = full ] || lib=boringssl_amd/csrc/build/$v/libbssl_amd.so
  export BSSL_AMD_LIB=$lib
  step c2_${v}_fetch 120 rocprofv3 --kernel-include-regex gcm_kernel --pmc FETCH_SIZE -d $O/c2_${v}_fetch -o run --output-format csv -- $B2
  step c2_${v}_write 120 rocprofv3 --kernel-include-regex gcm_kernel --pmc WRITE_SIZE -d $O/c2_${v}_write -o run --output-format csv -- $B2
  step c2_${v}_rdreq 120 rocprofv3 --kernel-include-regex gcm_kernel --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/c2_${v}_rdreq -o run --output-format csv -- $B2
done
unset BSSL_AMD_LIB
for cfg in config4 config5; do
  step stats_$cfg 600 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline
  B="python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline"
  step pmc_${cfg}_fetch 300 rocprofv3 --kernel-include-regex gcm_kernel --pmc FETCH_SIZE -d $O/pmc_${cfg}_fetch -o run --output-format csv -- $B
  step pmc_${cfg}_write 300 rocprofv3 --kernel-include-regex gcm_kernel --pmc WRITE_SIZE -d $O/pmc_${cfg}_write -o run --output-format csv -- $B
  step pmc_${cfg}_sq 300 rocprofv3 --kernel-include-regex gcm_kernel --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $O/pmc_${cfg}_sq -o run --output-format csv -- $B
done
