#!/bin/bash
# Round 5, session 9: table-free engine with quad LDS parking and lane values
# recomputed per use (fewer scratch round trips), and the L2 prefetch of each
# chunk's record bytes NR - k rounds before its output pass (BS_PF = k):
# parity of the product build, then same-box config 2 lines of HEAD, the
# product build (no prefetch) and k = 3 / 5 / 7, then configs G and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s9}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)" | tee -a $O/steps.log
  [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
}
export BSSL_AMD_GCM_MODE=bs
step pytest_bs 400 python -u -m pytest tests/test_gpu_parity.py -k "bitsliced or mix_kernel" -x -q --timeout 120 --timeout-method thread
step pytest_bs_total 500 python -u -m pytest tests/test_bs16_total.py -x -q --timeout 200 --timeout-method thread
L=boringssl_amd/csrc/build
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --config"
for v in base head pf3 pf5 pf7 base; do
  if [ $v = base ]; then step c2_$v 200 $B config2; else step c2_$v 200 env BSSL_AMD_LIB=$L/ab_$v/libbssl_amd.so $B config2; fi
done
for cfg in configG config4; do
  step ${cfg}_base 200 $B $cfg
  step ${cfg}_pf5 200 env BSSL_AMD_LIB=$L/ab_pf5/libbssl_amd.so $B $cfg
  step ${cfg}_pf3 200 env BSSL_AMD_LIB=$L/ab_pf3/libbssl_amd.so $B $cfg
done
