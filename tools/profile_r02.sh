#!/bin/bash
# Round-2 evidence on one GPU, into gpurun_out/r02/: for configs 2-5 the
# rocprofv3 kernel stats of the bench command and the PMC passes (FETCH_SIZE,
# WRITE_SIZE and the SQ/GRBM busy counters, each its own run), the bitsliced
# GCM mode's stats, and the FETCH/WRITE calibration copies of
# tools/micro/calib_copy.  Each GPU step has its own limit; the chain stops at
# the first failure.  Summarise with tools/pmc_traffic.py gpurun_out/r02.
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
for cfg in ${CONFIGS:-config2 config3 config4 config5}; do
  case $cfg in config3|config3x) K=chacha_poly_kernel ;; configS) K=gcm_siv_kernel ;; *) K=gcm_kernel ;; esac
  step stats_$cfg 300 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
  B="python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline"
  step pmc_${cfg}_fetch 200 rocprofv3 --kernel-include-regex $K --pmc FETCH_SIZE -d $O/pmc_${cfg}_fetch -o run --output-format csv -- $B
  step pmc_${cfg}_write 200 rocprofv3 --kernel-include-regex $K --pmc WRITE_SIZE -d $O/pmc_${cfg}_write -o run --output-format csv -- $B
  step pmc_${cfg}_sq 200 rocprofv3 --kernel-include-regex $K --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $O/pmc_${cfg}_sq -o run --output-format csv -- $B
done
if [ -z "${CONFIGS:-}" ]; then
  BSSL_AMD_GCM_MODE=bs step stats_config2_bs 300 rocprofv3 --kernel-trace --stats -d $O/prof_config2_bs -o run \
    --output-format csv -- python3 bench.py --config config2 --steps 10 --warmup 2 --no-cpu-baseline
  step calib_run 60 tools/micro/calib_copy 5
  step calib_fetch 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- tools/micro/calib_copy 2
  step calib_write 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- tools/micro/calib_copy 2
fi
