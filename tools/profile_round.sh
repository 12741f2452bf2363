#!/bin/bash
# Round-end evidence on one GPU: rocprofv3 kernel stats of the bench command
# for config2 (headline) and config3, and the HBM-traffic PMC passes
# (separate FETCH_SIZE / WRITE_SIZE runs, MI355X_MICROARCH.md HBM section)
# at the full bench size.  Output: gpurun_out/prof_<cfg>/, gpurun_out/pmc_<cfg>_*.
# Each GPU step has its own time limit and the chain stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/profile_steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/profile_steps.log
  [ $rc -eq 0 ] || exit $rc
}
for cfg in ${CONFIGS:-config2 config3}; do
  case $cfg in config3|config3x) K=chacha_poly_kernel ;; configS) K=gcm_siv_kernel ;; *) K=gcm_kernel ;; esac
  step "stats_$cfg" 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$cfg" -o run \
    --output-format csv -- python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu-baseline
  B="python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline"
  step "pmc_${cfg}_fetch" 300 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE \
    -d "gpurun_out/pmc_${cfg}_fetch" -o run --output-format csv -- $B
  step "pmc_${cfg}_write" 300 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE \
    -d "gpurun_out/pmc_${cfg}_write" -o run --output-format csv -- $B
  step "pmc_${cfg}_sq" 300 rocprofv3 --kernel-include-regex "$K" --pmc SQ_LDS_IDX_ACTIVE \
    SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES \
    GRBM_GUI_ACTIVE -d "gpurun_out/pmc_${cfg}_sq" -o run --output-format csv -- $B
done
