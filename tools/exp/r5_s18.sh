#!/bin/bash
# Round 5, session 18: E_K(J0) production at s_setprio 3: per-group timing,
# parity, configs 2 / G / 4 / 5 of the table-free engine.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s18}
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
step prof 200 env BSSL_AMD_LIB=boringssl_amd/csrc/build/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config config2
grep "bs_grp groups\|bs_prof" $O/prof.log | tail -2
step pytest_bs 400 python -u -m pytest tests/test_gpu_parity.py -k "bitsliced or mix_kernel" -x -q --timeout 120 --timeout-method thread
for cfg in config2 configG config4 config5; do
  step ${cfg}_bs 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
done
step pytest_bs_total 500 python -u -m pytest tests/test_bs16_total.py -x -v --timeout 200 --timeout-method thread
