#!/bin/bash
# Round 5, session 5: where the fused table-free engine's time goes on
# config 2 -- ablation builds of gcm_bs.hip (BSSL_AMD_BS_ABLATE: 1 output pass
# without the GHASH multiply, 2 without the record loads/stores, 3 neither,
# 4 no output pass at all) against the full engine, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r5s5
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -1 "$O/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
export BSSL_AMD_GCM_MODE=bs
B="python bench.py --config config2 --steps 10 --warmup 2 --no-cpu-baseline --no-parity"
L=boringssl_amd/csrc/build
step bs 200 $B
for n in 1 2 3 4; do step abl$n 200 env BSSL_AMD_LIB=$L/ab_bsa$n/libbssl_amd.so $B; done
step bs_2 200 $B
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
export BSSL_AMD_LIB=$L/ab_bsa4/libbssl_amd.so
step pmc_abl4 200 rocprofv3 --kernel-include-regex gcm_bs_kernel --pmc $PMC -d $O/pmc_abl4 -o run --output-format csv -- \
  python3 bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity
