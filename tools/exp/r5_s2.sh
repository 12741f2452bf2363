#!/bin/bash
# Round 5, session 2: first run of the fused table-free engine (gcm_bs.hip):
# its GPU parity suite, then same-box bench lines of both engines on config 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s2}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -3 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
#step pytest_bs 400 python -u -m pytest tests/test_gpu_parity.py -k "bitsliced or mix_kernel" -x -q --timeout 120 --timeout-method thread
step pytest_bs_total 500 python -u -m pytest tests/test_bs16_total.py -x -q --timeout 200 --timeout-method thread
B="python bench.py --config config2 --steps 10 --warmup 2 --no-cpu-baseline"
step table 200 env BSSL_AMD_GCM_MODE=table $B
step bs 200 env BSSL_AMD_GCM_MODE=bs $B
step table_2 200 env BSSL_AMD_GCM_MODE=table $B --no-parity
step bs_2 200 env BSSL_AMD_GCM_MODE=bs $B --no-parity
export BSSL_AMD_GCM_MODE=bs
step stats_bs 300 rocprofv3 --kernel-trace --stats -d $O/stats_bs -o run --output-format csv -- \
  python3 bench.py --config config2 --steps 5 --warmup 1 --no-cpu-baseline --no-parity
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
step pmc_bs 200 rocprofv3 --kernel-include-regex gcm_bs_kernel --pmc $PMC -d $O/pmc_bs -o run --output-format csv -- \
  python3 bench.py --config config2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity
