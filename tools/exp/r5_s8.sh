#!/bin/bash
# Round 5, session 8: where the table-free engine's wave time goes on config 2
# -- the phase-clock build (BSSL_AMD_BS_PROF: s_memtime laps per chunk phase),
# then SQ / SQC counter passes of the product kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s8}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -2 "$O/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
export BSSL_AMD_GCM_MODE=bs
L=boringssl_amd/csrc/build
B="python bench.py --config config2 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
step prof 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so $B
step bs 200 $B
P="--config config2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity"
PMC1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc1 120 rocprofv3 --kernel-include-regex gcm_bs_kernel --pmc $PMC1 -d $O/pmc1 -o run --output-format csv -- python3 bench.py $P
PMC2="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
step pmc2 120 rocprofv3 --kernel-include-regex gcm_bs_kernel --pmc $PMC2 -d $O/pmc2 -o run --output-format csv -- python3 bench.py $P
step pytest_keys 300 python -u -m pytest tests/test_key_setup.py tests/test_aead_api_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step keysetup 200 python -u tools/keysetup_bench.py
