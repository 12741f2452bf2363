#!/bin/bash
# Round 5, session 1: where the bs16 engine's time goes on config 2 --
# same-box bench lines of the T-table and bs16 engines, the bs16 ablation
# builds (BSSL_AMD_BS16_ABLATE: 1 no GHASH, 2 no record I/O, 3 neither,
# 4 no output transposes, 7 rounds + round-0 only), kernel stats and one
# SQ/GRBM PMC pass of the bs16 kernel and of ablation 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r5s1
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -1 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
B="python bench.py --config config2 --steps 10 --warmup 2 --no-cpu-baseline --no-parity"
L=boringssl_amd/csrc/build
step table 200 $B
step bs16 200 env BSSL_AMD_GCM_MODE=bs16 $B
for n in 1 2 3 4 7; do
  step bs16_abl$n 200 env BSSL_AMD_GCM_MODE=bs16 BSSL_AMD_LIB=$L/ab_bsabl$n/libbssl_amd.so $B
done
step table_2 200 $B
step bs16_2 200 env BSSL_AMD_GCM_MODE=bs16 $B
export BSSL_AMD_GCM_MODE=bs16
step stats_bs16 300 rocprofv3 --kernel-trace --stats -d $O/stats_bs16 -o run --output-format csv -- \
  python3 bench.py --config config2 --steps 5 --warmup 1 --no-cpu-baseline --no-parity
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
step pmc_bs16 200 rocprofv3 --kernel-include-regex gcm_bs16_kernel --pmc $PMC -d $O/pmc_bs16 -o run --output-format csv -- \
  python3 bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity
export BSSL_AMD_LIB=$L/ab_bsabl3/libbssl_amd.so
step pmc_abl3 200 rocprofv3 --kernel-include-regex gcm_bs16_kernel --pmc $PMC -d $O/pmc_abl3 -o run --output-format csv -- \
  python3 bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity
