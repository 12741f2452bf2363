#!/bin/bash
# Round 5, session 15: E_K(J0) produced kBsAhead groups ahead (the first
# kBsAhead groups by units 0..kBsAhead-1 in parallel), s_setprio 2 output pass:
# parity, phase clocks, configs 2 / G / 4 / 5, same-box A/B of the distance.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s15}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1) $(grep -o 'ref_digest_[a-z]*' $O/$name.log | head -1)" | tee -a $O/steps.log
  [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
}
export BSSL_AMD_GCM_MODE=bs
step pytest_bs 400 python -u -m pytest tests/test_gpu_parity.py -k "bitsliced or mix_kernel" -x -q --timeout 120 --timeout-method thread
L=boringssl_amd/csrc/build
for cfg in config2 configG; do
  step prof_$cfg 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config $cfg
  grep bs_prof $O/prof_$cfg.log | tail -1
done
for cfg in config2 configG config4 config5; do
  step ${cfg}_bs 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
  step ${cfg}_a2 200 env BSSL_AMD_LIB=$L/ab_ahead2/libbssl_amd.so python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-parity
  step ${cfg}_a8 200 env BSSL_AMD_LIB=$L/ab_ahead8/libbssl_amd.so python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-parity
done
step pytest_bs_total 500 python -u -m pytest tests/test_bs16_total.py -x -v --timeout 200 --timeout-method thread
